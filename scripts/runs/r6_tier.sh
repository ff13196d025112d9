#!/bin/bash
# The GPU test tier (as the driver runs it) plus smoke(), on the current build.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/tier
mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/tier.log 2>&1
rc=$?; tail -5 $out/tier.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -2 $out/smoke.log
