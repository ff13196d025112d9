#!/bin/bash
# Kernel trace of the emulated p = 8 rank at N = 16384, comm-free (chain / MAIN per step).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/temu
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 > $o/emu.log 2>&1 || { tail -5 $o/emu.log; exit 1; }
cat $o/emu.log
python3 scripts/side_chain.py $o/prof/run_results.db 128 2 > $o/side.md; cat $o/side.md
