#!/bin/bash
# Round 6: panel-blocked (one workgroup per candidate) vs the GPU-wide form at large m, few / more
# candidates (bench/bench_blockinv.py: device time per batch, 3 batches each).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/bilarge
mkdir -p $out
for m in 512 1024 2048 4096; do
  for v in huge panel; do
    BI_M="$m" BI_NBLK="2 8" BI_REPS=3 timeout -k 10 200 python3 bench/bench_blockinv.py $v >> $out/bi2.jsonl 2>> $out/bi2.err || { tail -5 $out/bi2.err; exit 1; }
    tail -4 $out/bi2.jsonl
  done
done
