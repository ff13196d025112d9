#!/bin/bash
# Round 6: kernel trace of the N = 8192 solve (closing build) and the pivot-chain breakdown.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/trace8k
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --size 8192 --steps 3 --warmup 1 > $out/prof.log 2>&1 || exit $?
tail -1 $out/prof.log | cut -c1-200
db=$(find $out/prof -name "*.db" | head -1)
python3 scripts/rocpd_summary.py $db "N = 8192, round-6 closing build" > $out/summary.md 2>&1 || exit $?
python3 scripts/side_chain.py $db 64 2 > $out/chain.md 2>&1 || exit $?
tail -30 $out/chain.md
