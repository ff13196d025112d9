#!/bin/bash
# rocprofv3 kernel trace of the lazy pair schedule (GJ_LAZY=1) at N = 32768: MAIN gaps, kernel table.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_lazy
mkdir -p $out
GJ_LAZY=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $out -o run -- python3 bench.py --steps 1 --warmup 1 --no-residual > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
db=$(find $out -name "*.db" | head -1)
python3 scripts/main_gaps.py "$db" > gpurun_out/prof_lazy_gaps.txt 2>&1 || exit 1
python3 scripts/rocpd_summary.py "$db" > gpurun_out/prof_lazy_summary.md 2>&1 || exit 1
head -22 gpurun_out/prof_lazy_gaps.txt; head -16 gpurun_out/prof_lazy_summary.md; tail -8 gpurun_out/prof_lazy_summary.md
