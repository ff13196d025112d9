#!/bin/bash
# rocprofv3 kernel trace of the p-rank emulation (rank 0 of a p-GPU job alone on one GPU) and
# the pivot-chain breakdown of its SIDE stream.   bash scripts/prof_emu.sh <tag> <p> <N>
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$1
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out" -o run -- python3 bench/bench_emulate.py --ranks $2 --size $3 --reps 1 > "$out/emu.log" 2>&1 || exit 1
db=$(find "$out" -name "*.db" | head -1)
python3 scripts/side_chain.py "$db" $(( $3 / 128 ))
