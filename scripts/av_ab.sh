#!/bin/bash
# LDS-DMA GEMM with A direct to VGPRs (GJ_GLDS_AV=1: 3 WG/CU, 2: 4 WG/CU) vs A through LDS (0).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for av in 1 2; do
  GJ_GLDS_AV=$av timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "glds or auto" --timeout 120 --timeout-method thread > gpurun_out/av_tests.log 2>&1 || { tail -20 gpurun_out/av_tests.log; exit 1; }
  tail -1 gpurun_out/av_tests.log
done
for rep in 1 2; do
  for av in 0 1 2; do
    for shape in "32768 8192 512" "4096 32768 1024"; do
      GJ_GLDS_AV=$av timeout -k 10 60 python bench/gemm_probe.py $shape --variant glds 2>&1 | grep -v amdgpu.ids | sed "s/^/av=$av /" || exit 1
    done
  done
done
for av in 0 1 2; do
  GJ_GLDS_AV=$av timeout -k 10 200 python bench.py --size 32768 --steps 3 --no-residual > gpurun_out/av.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/av.json "av=$av n=32768" || exit 1
done
