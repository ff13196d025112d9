#!/bin/bash
# Round 6: the driver's headline command under a clock/power sampler, plus the fixed MFMA peak
# probe (burst + 20 s sustained).  profiles/sustained_r6.md.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/sus
mkdir -p $out
timeout -k 10 120 build/mfma_peak 20 > $out/peak.jsonl 2> $out/peak.err || exit $?
timeout -k 10 300 python3 scripts/smi_sample.py $out/smi_32768.jsonl -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/b32768.json 2> $out/b32768.err || exit $?
timeout -k 10 120 python3 bench.py --size 8192 > $out/b8192.json 2> $out/b8192.err || exit $?
timeout -k 10 120 python3 bench.py --size 16384 > $out/b16384.json 2> $out/b16384.err || exit $?
tail -2 $out/peak.jsonl; cut -c1-400 $out/b32768.json
