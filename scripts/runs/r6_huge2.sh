#!/bin/bash
# Round 6: the live-count rule between the panel-blocked and GPU-wide candidate inverses: kernel
# and engine tests of the large-block paths.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/huge2
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
    -k "huge or large_m or pivot_rule or block_size_above" > $out/kern.log 2>&1; rc=$?; tail -4 $out/kern.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_engine.py \
    -k "large_blocks" > $out/eng.log 2>&1; rc=$?; tail -4 $out/eng.log; exit $rc
