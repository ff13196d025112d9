#!/bin/bash
# p = 8 ranks (4096 rows, 32 reserved CUs -> 224 x 4 GEMM slots): chunk widths whose tile count is a
# multiple of the resident slots (7168 / 5376 / 3584) against the default 8192.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for c in 8192 7168 5376 3584 8192 7168; do
  timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 2 --bw 100 --chunk-cols $c > gpurun_out/p8q.log 2>&1 || { tail -5 gpurun_out/p8q.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/p8q.log | sed "s/^/chunk=$c /"
done | tee gpurun_out/p8_chunk_quant.log
