#!/bin/bash
# Round 6: kernel trace of the N = 32768 solve (final build) and the pivot-chain breakdown.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/trace32k
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 2 --warmup 1 > $out/prof.log 2>&1 || exit $?
tail -1 $out/prof.log | cut -c1-200
db=$(find $out/prof -name "*.db" | head -1)
python3 scripts/rocpd_summary.py $db "N = 32768, round-6 final build" > $out/summary.md 2>&1 || exit $?
python3 scripts/side_chain.py $db 256 4 > $out/chain.md 2>&1 || exit $?
tail -30 $out/chain.md
