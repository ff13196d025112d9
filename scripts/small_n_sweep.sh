#!/bin/bash
# Small-N (side-chain-bound) configurations: block size x panel depth at N (default 8192).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for cfg in ${CFGS:-"128 4" "128 2" "64 8" "64 4" "128 8"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --size ${N:-8192} --block $1 --depth $2 --steps 5 --warmup 2 > gpurun_out/sn_$1_$2.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('m', sys.argv[2], 'depth', sys.argv[3], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/sn_$1_$2.json $1 $2 || exit 1
done
