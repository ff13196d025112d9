#!/bin/bash
# A/B on one box: ab/old (previous build, copied package + bench.py) vs the tree, interleaved.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for s in ${SIZES:-8192 16384}; do
  for r in 1 2; do
    for v in old new; do
      b=bench.py; [ $v = old ] && b=ab/old/bench.py
      timeout -k 10 200 python $b --size $s --steps 5 --warmup 2 --no-residual > gpurun_out/ab_${v}_${s}_$r.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms')" gpurun_out/ab_${v}_${s}_$r.json $v || exit 1
    done
  done
done
