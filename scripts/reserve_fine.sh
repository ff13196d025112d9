#!/bin/bash
# Finer CU-reservation sweep at the pivot-chain-bound sizes (bench.py, 3 timed inversions).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in 8192 16384; do
  for rc in 16 24 32 40 48; do
    GJ_RESERVE_CUS=$rc timeout -k 10 120 python bench.py --size $n --steps 3 --no-residual > gpurun_out/rf.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/rf.json "n=$n reserve=$rc" || exit 1
  done
done
