#!/bin/bash
# GPU tier (full), then the round-4 measurements (scripts/runs/r4_measure.sh) if the tier did not crash.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests.txt 2>&1
rc=$?; echo "tests_rc=$rc" >> gpurun_out/gputests.txt; tail -4 gpurun_out/gputests.txt
[ $rc -le 1 ] || exit $rc
bash scripts/runs/r4_measure.sh
