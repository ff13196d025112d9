#!/bin/bash
# Broadcast/GEMM chunk width sweep in the p-rank critical-path emulation (and the real 1-GPU solve).
#   CHUNKS="8192 6144" RANKS="2 4 8" bash scripts/chunk_sweep.sh
cd "$(dirname "$0")/.." || exit 1
for cc in ${CHUNKS:-8192 6144}; do
  echo "chunk_cols=$cc"
  timeout -k 10 400 python bench/bench_emulate.py --ranks ${RANKS:-2 4 8} --reps 2 --chunk-cols $cc 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-residual --chunk-cols $cc 2>/dev/null || exit 1
done
