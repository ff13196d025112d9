#!/bin/bash
# fp64 block size 256 vs 128 at the headline size (depth = steps fused per trailing update).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for cfg in "128 4" "256 2" "256 4" "192 2" "192 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --size ${SIZE:-32768} --block $1 --depth $2 > gpurun_out/m_sweep_$1_$2.json 2>gpurun_out/m_sweep_$1_$2.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('m', d['config']['m'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', d['value'], 'GFLOP/s', d['residual_inf'])" gpurun_out/m_sweep_$1_$2.json || exit 1
done
