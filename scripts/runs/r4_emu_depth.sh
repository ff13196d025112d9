#!/bin/bash
# Depth 4 vs 8 on the p = 2 / 4 ranks of N = 32768 (co-resident inverse, no reservation), rank-0
# emulation under the 50 GB/s direct-broadcast model.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/emudepth
mkdir -p $o
timeout -k 10 600 python bench/bench_emulate.py --ranks 2 4 --size 32768 --depth 4 8 --reps 2 --bw 50 --bcast direct > $o/emu.txt 2>&1 || exit $?
grep '"seconds"' $o/emu.txt
