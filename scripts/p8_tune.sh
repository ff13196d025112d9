#!/bin/bash
# p = 8 rank emulation at N = 32768 under the cost model (100 GB/s): depth x chunk width.
cd "$(dirname "$0")/.." || exit 1
for d in 3 4 6 8; do
  for cc in 4096 8192; do
    timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 2 --depth $d --chunk-cols $cc --bw ${BW:-100} 2>&1 | grep -v amdgpu.ids | sed "s/^/depth=$d chunk=$cc /" || exit 1
  done
done
