#!/bin/bash
# Tile-walk group size at the p = 8 trailing-update shapes (4096-row ranks, K = 1024).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for shape in "4096 8192 1024" "4096 32768 1024" "8192 8192 512"; do
  for g in 1 2 4 8 16 32; do
    GJ_GEMM_GROUP=$g timeout -k 10 60 python bench/gemm_probe.py $shape --variant glds | sed "s/^/g=$g /" || exit 1
  done
  for g in 4 16; do
    GJ_GEMM_GROUP=$g timeout -k 10 60 python bench/gemm_probe.py $shape --variant dtva | sed "s/^/g=$g /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/group_p8.log
