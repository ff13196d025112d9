#!/bin/bash
# Panel depth 3 against the engine's choice (2 up to N = 8192, 4 above).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for s in 8192 16384; do
  for r in 1 2; do
    for d in 0 3; do
      timeout -k 10 200 python bench.py --size $s --depth $d --steps 5 --warmup 2 --no-residual > gpurun_out/d3_${d}_${s}_$r.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('N', d['config']['n'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms')" gpurun_out/d3_${d}_${s}_$r.json || exit 1
    done
  done
done
