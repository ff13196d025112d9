#!/bin/bash
# Quick GPU iteration: block-inverse tests + microbench, full GPU test suite, p-rank emulation.
# Every GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k block_inverse > gpurun_out/bi_test.log 2>&1 || exit $?
timeout -k 10 300 python bench/bench_blockinv.py > gpurun_out/bi.log 2>&1 || exit $?
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/gt.log 2>&1 || exit $?
timeout -k 10 300 python bench/bench_emulate.py --ranks 1 4 8 > gpurun_out/emu.log 2>&1 || exit $?
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 --size 16384 >> gpurun_out/emu.log 2>&1 || exit $?
