#!/bin/bash
# fp64 LDS-DMA GEMM: LDS reads drained before the slice barrier (0) vs not (GJ_GEMM_ABLATE=2);
# then BASELINE config 5 (fp32 N=65536) with the fp32 LDS-DMA kernel
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "glds or gemm" --timeout 120 --timeout-method thread > gpurun_out/lgkm_tests.log 2>&1 || { tail -30 gpurun_out/lgkm_tests.log; exit 1; }
tail -1 gpurun_out/lgkm_tests.log
for rep in 1 2; do
for ab in "" 1; do
  for shape in "32768 8192 512" "4096 32768 1024"; do
    env ${ab:+GJ_GLDS_NODRAIN=1} timeout -k 10 60 python bench/gemm_probe.py $shape --variant auto 2>&1 | grep -v amdgpu.ids | sed "s/^/ab=$ab /" || exit 1
  done
  env ${ab:+GJ_GLDS_NODRAIN=1} timeout -k 10 200 python bench.py --size 32768 --steps 3 --no-residual > gpurun_out/lg.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/lg.json "ab=$ab n=32768" || exit 1
done
done
timeout -k 10 300 python bench.py --size 65536 --dtype fp32 --steps 2 > gpurun_out/f32_65536.json 2>/dev/null || exit 1
cat gpurun_out/f32_65536.json
