#!/bin/bash
# depth (steps fused per trailing update) at p = 1 (bench.py) and emulated p = 2 / 4 (cost model 100 GB/s)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in 16384 32768; do
  for d in 4 6 8; do
    timeout -k 10 200 python bench.py --size $n --depth $d --steps 3 --no-residual > gpurun_out/dt.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/dt.json "p=1 n=$n depth=$d" || exit 1
  done
done
for p in 2 4; do
  for d in 4 6 8; do
    timeout -k 10 300 python bench/bench_emulate.py --ranks $p --size 32768 --reps 2 --depth $d --bw 100 2>&1 | grep -v amdgpu.ids | sed "s/^/depth=$d /" || exit 1
  done
done
for d in 4 6 8; do
  timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 16384 --reps 2 --depth $d --bw 100 2>&1 | grep -v amdgpu.ids | sed "s/^/depth=$d /" || exit 1
done
