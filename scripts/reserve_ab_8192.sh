#!/bin/bash
# CU reservation at N = 8192 with the small COMM tiles (GJ_RESERVE_CUS, first-CUs mask).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for c in 32 16 48 64; do
    GJ_RESERVE_CUS=$c GJ_RESERVE_MODE=0 timeout -k 10 200 python bench.py --size 8192 --steps 5 --warmup 2 --no-residual > gpurun_out/rs_${c}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('reserve', sys.argv[2], d['ms_per_step'], 'ms')" gpurun_out/rs_${c}_$r.json $c || exit 1
  done
done
