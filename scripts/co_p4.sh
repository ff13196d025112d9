#!/bin/bash
# Co-resident candidate inverse (GJ_BI_VARIANT=co) at the p = 2 / 4 rank shapes of N = 32768, where
# the pivot chain waits for whole CUs (no reservation): rank-0 emulation, 100 GB/s model.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in panel co panel co; do
  GJ_BI_VARIANT=$v timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 --size 32768 --reps 2 --bw 100 > gpurun_out/co4.log 2>&1 || { tail -5 gpurun_out/co4.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/co4.log | sed "s/^/bi=$v /" | cut -c1-150
done | tee gpurun_out/co_p4.log
