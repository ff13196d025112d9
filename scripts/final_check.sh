#!/bin/bash
# Round-end style check on one GPU: the GPU test tier, then bench.py at the BASELINE sizes.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || exit 1
tail -1 gpurun_out/gpu_tests_final.log
for s in ${SIZES:-8192 16384 32768}; do
  timeout -k 10 200 python bench.py --size $s > gpurun_out/bench_final_$s.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', d['value'], 'GFLOP/s', d['residual_inf'])" gpurun_out/bench_final_$s.json || exit 1
done
