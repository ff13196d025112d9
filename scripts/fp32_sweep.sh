#!/bin/bash
# fp32 65536 (BASELINE config 5): block size x panel depth.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for cfg in ${CFGS:-"128 4" "128 8" "256 4" "256 2"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --size ${N:-65536} --dtype fp32 --block $1 --depth $2 --steps 2 --warmup 1 --no-residual > gpurun_out/fp32_$1_$2.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('m', sys.argv[2], 'depth', sys.argv[3], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF')" gpurun_out/fp32_$1_$2.json $1 $2 || exit 1
done
