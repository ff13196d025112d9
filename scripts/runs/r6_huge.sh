#!/bin/bash
# Round 6: the GPU-wide candidate inverse for m > 4096 (kernel tests, then the solver at m = 5000 /
# 4500), one step at a time under its own time limit.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/huge
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
    -k "huge and not engine" > $out/kern.log 2>&1; rc=$?; tail -15 $out/kern.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
    -k "block_size_above_4096" > $out/eng.log 2>&1; rc=$?; tail -8 $out/eng.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/gj --gen random 8192 8192 > $out/gj8192.log 2> $out/gj8192.err; rc=$?; tail -4 $out/gj8192.log; exit $rc
