#!/bin/bash
# rocprofv3 trace of the p = 4 rank-0 emulation at N = 32768: SIDE-chain breakdown and MAIN gaps.
cd "$(dirname "$0")/.." || exit 1
bash scripts/prof_emu.sh emu4r2 4 32768 > gpurun_out/prof_emu4r2_side.txt 2>&1 || exit 1
db=$(find gpurun_out/prof_emu4r2 -name "*.db" | head -1)
python3 scripts/main_gaps.py "$db" > gpurun_out/prof_emu4r2_gaps.txt 2>&1 || exit 1
python3 scripts/rocpd_summary.py "$db" > gpurun_out/prof_emu4r2_summary.md 2>&1 || exit 1
head -16 gpurun_out/prof_emu4r2_side.txt; head -24 gpurun_out/prof_emu4r2_gaps.txt
