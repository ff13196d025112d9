#!/bin/bash
# Where the fp64 GEMM plateau comes from: C traffic (acc vs store, deep K) and tile order (group).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in glds dtva; do
  for g in 1 4 8 16; do
    GJ_GEMM_GROUP=$g timeout -k 10 60 python bench/gemm_probe.py 32768 8192 512 --variant $v | sed "s/^/g=$g /" || exit 1
  done
  timeout -k 10 60 python bench/gemm_probe.py 32768 8192 512 --variant $v --op store || exit 1
  timeout -k 10 60 python bench/gemm_probe.py 32768 8192 2048 --variant $v || exit 1
  timeout -k 10 60 python bench/gemm_probe.py 32768 8192 4096 --variant $v --reps 10 || exit 1

done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/dtva_probe2.log
timeout -k 10 120 python bench/bench_vendor_gemm.py 2>&1 | grep -v amdgpu.ids | grep float64 | tee -a gpurun_out/dtva_probe2.log
