#!/bin/bash
# N = 8192 kernel trace of the current build (chain / chunk pass / MAIN per step).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/t8k
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --size 8192 --steps 5 --warmup 2 --no-residual > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
python3 scripts/side_chain.py $o/prof/run_results.db > $o/side.md; head -16 $o/side.md
