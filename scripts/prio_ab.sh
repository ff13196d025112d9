#!/bin/bash
# s_setprio(1) around the MFMA clusters of the LDS-DMA kernels (GJ_GLDS_STAGES=90 / GJ_GLDS32=90)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
GJ_GLDS_STAGES=90 GJ_GLDS32=90 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "glds or deep_auto" --timeout 120 --timeout-method thread > gpurun_out/prio_tests.log 2>&1 || { tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
for rep in 1 2; do
for c in 9 90; do
  for shape in "32768 8192 512" "4096 32768 1024"; do
    GJ_GLDS_STAGES=$c timeout -k 10 60 python bench/gemm_probe.py $shape --variant auto 2>&1 | grep -v amdgpu.ids | sed "s/^/f64 c=$c /" || exit 1
  done
done
for c in 0 90; do
  for shape in "32768 16384 512" "4096 65536 1024"; do
    GJ_GLDS32=$c timeout -k 10 60 python bench/gemm_probe.py $shape --dtype fp32 --variant auto 2>&1 | grep -v amdgpu.ids | sed "s/^/f32 c=$c /" || exit 1
  done
done
done
