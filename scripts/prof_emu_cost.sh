#!/bin/bash
# rocprofv3 kernel trace of the p-rank emulation WITH the communication-cost model, then the
# pivot-chain (SIDE) breakdown and the MAIN-stream idle gaps.   bash scripts/prof_emu_cost.sh <tag> <p> <N> <bw>
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$1
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out" -o run -- python3 bench/bench_emulate.py --ranks $2 --size $3 --reps 1 --bw $4 > "$out/emu.log" 2>&1 || exit 1
db=$(find "$out" -name "*.db" | head -1)
python3 scripts/side_chain.py "$db" $(( $3 / 128 )) > "$out/side_chain.md" || exit 1
python3 scripts/main_gaps.py "$db" > "$out/main_gaps.md" || exit 1
grep -v amdgpu.ids "$out/emu.log"; cat "$out/side_chain.md" "$out/main_gaps.md"
