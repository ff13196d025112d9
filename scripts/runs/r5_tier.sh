#!/bin/bash
# Whole GPU tier on the current build, then smoke().
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/tier
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputests.txt 2>&1
rc=$?
tail -3 $o/gputests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.txt 2>&1 || { tail -5 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
