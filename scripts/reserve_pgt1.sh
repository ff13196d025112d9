#!/bin/bash
# CU reservation at p > 1 under the communication-cost model (rank-0 emulation, N = 32768):
# 0 vs 32 CUs kept off the trailing update, comm-free and at 50 / 100 GB/s.
cd "$(dirname "$0")/.." || exit 1
for p in 2 4 8; do
  for rc in 0 32; do
    GJ_RESERVE_CUS=$rc timeout -k 10 300 python bench/bench_emulate.py --ranks $p --size ${SIZE:-32768} --reps 2 --bw 50 100 2>&1 | grep -v amdgpu.ids | sed "s/^/reserve=$rc /" || exit 1
  done
done
