#!/bin/bash
# Kernel traces of the small-N cases: N = 8192 on one GPU, and rank 0 of the emulated p = 4,
# N = 16384 job (BASELINE config 3), comm-free.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r3_8192 gpurun_out/prof_r3_emu4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3_8192 -o run -- \
    python3 bench.py --size 8192 --steps 2 --warmup 1 --no-residual > gpurun_out/prof_r3_8192/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3_emu4 -o run -- \
    python3 bench/bench_emulate.py --ranks 4 --size 16384 --reps 1 > gpurun_out/prof_r3_emu4/emu.log 2>&1
