#!/bin/bash
# A/B of HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the launch-bound pivot chain.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for s in ${SIZES:-8192 16384 32768}; do
  for r in 1 2; do
    for v in 0 1; do
      HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --size $s --steps 5 --warmup 2 --no-residual > gpurun_out/ka_${v}_${s}_$r.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('kernarg', sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms')" gpurun_out/ka_${v}_${s}_$r.json $v || exit 1
    done
  done
done
