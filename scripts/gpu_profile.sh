#!/bin/bash
# rocprofv3 kernel trace + stats of one bench step (no PMC counters in this run).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/prof_${1:-default}
shift
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out" -o run -- python3 bench.py "$@" > "$out/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$out/bench.log"
find "$out" -name "*stats*" | head
exit $rc
