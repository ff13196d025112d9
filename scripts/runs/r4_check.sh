#!/bin/bash
# Round 4 GPU check: the GPU test tier, then (only if it did not time out / crash) a short headline
# bench and a kernel-trace profile of two N = 32768 inversions.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.txt 2>&1
rc=$?; echo "tests_rc=$rc" >> gpurun_out/gputests.txt; tail -3 gpurun_out/gputests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.txt 2>&1
rc=$?; tail -1 gpurun_out/bench1.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh r4 --steps 2 --warmup 1 --no-residual
