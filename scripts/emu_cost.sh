#!/bin/bash
# p-rank emulation with ShadowComm's communication-cost model (bench/bench_emulate.py --bw):
# comm-free baseline + modelled transfer time at several algorithm bandwidths.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in ${SIZES:-32768 16384}; do
  timeout -k 10 400 python bench/bench_emulate.py --ranks 2 4 8 --size $n --reps 1 --bw ${BWS:-50 100 200} --lat ${LAT:-20} > gpurun_out/emu_cost_$n.log 2>&1 || { tail -5 gpurun_out/emu_cost_$n.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/emu_cost_$n.log
done
