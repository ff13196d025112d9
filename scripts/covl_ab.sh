#!/bin/bash
# C-tile load overlapped with the first LDS-DMA slice (GJ_GLDS_COVL=1, default) vs serialised (0).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for c in 0 1; do
    GJ_GLDS_COVL=$c timeout -k 10 60 python bench/gemm_probe.py 32768 8192 512 --variant glds --check 2>&1 | grep -v amdgpu.ids | sed "s/^/covl=$c /" || exit 1
    GJ_GLDS_COVL=$c timeout -k 10 60 python bench/gemm_probe.py 4096 32768 1024 --variant glds 2>&1 | grep -v amdgpu.ids | sed "s/^/covl=$c /" || exit 1
    GJ_GLDS_COVL=$c timeout -k 10 200 python bench.py --size 32768 --steps 3 --no-residual > gpurun_out/covl.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/covl.json "covl=$c n=32768" || exit 1
  done
done
