#!/bin/bash
# Round 6: the policy-cliff sweep on the final per-rank tile rule (profiles/policy_sweep_r6.md).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/sweep2
mkdir -p $out
timeout -k 10 1000 python3 scripts/policy_sweep.py $out/sweep.jsonl > $out/sweep.md 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 1; }
tail -24 $out/sweep.md
