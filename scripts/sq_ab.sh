#!/bin/bash
# 128 x 128 LDS-DMA tiles with slice depth 8 / 16 (GJ_GLDS_SQ=8 / 16 / 163 = 3 stages) vs 128 x 64 (0)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for sq in 8 16 163; do
  GJ_GLDS_SQ=$sq timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "glds" --timeout 120 --timeout-method thread > gpurun_out/sq_tests.log 2>&1 || { tail -20 gpurun_out/sq_tests.log; exit 1; }
  tail -1 gpurun_out/sq_tests.log
done
for sq in 0 8 16 163; do
  for shape in "32768 8192 512" "4096 32768 1024"; do
    GJ_GLDS_SQ=$sq timeout -k 10 60 python bench/gemm_probe.py $shape --variant glds 2>&1 | grep -v amdgpu.ids | sed "s/^/sq=$sq /" || exit 1
  done
done
for sq in 0 16; do
  GJ_GLDS_SQ=$sq timeout -k 10 200 python bench.py --size 32768 --steps 3 --no-residual > gpurun_out/sq.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/sq.json "sq=$sq n=32768" || exit 1
done
