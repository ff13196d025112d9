#!/bin/bash
# A-direct GEMM for the deep trailing updates (GJ_DEEP_DTVA=1) vs the LDS-DMA kernel: p-rank
# emulation under the 100 GB/s cost model, and one-GPU bench.py at 16384 / 32768.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in 0 1 0 1; do
  GJ_DEEP_DTVA=$v timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --reps 2 --bw 100 > gpurun_out/de.log 2>&1 || { tail -5 gpurun_out/de.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/de.log | grep model_bw | sed "s/^/dtva=$v /" | cut -c1-140
  GJ_DEEP_DTVA=$v timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --reps 2 --bw 100 > gpurun_out/de.log 2>&1 || { tail -5 gpurun_out/de.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/de.log | grep model_bw | sed "s/^/dtva=$v /" | cut -c1-140
  GJ_DEEP_DTVA=$v timeout -k 10 200 python bench.py --size 16384 --steps 5 > gpurun_out/de.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('dtva', sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms')" gpurun_out/de.json $v || exit 1
done 2>&1 | tee gpurun_out/dtva_emu.log
