#!/bin/bash
# Block-inverse iteration on one GPU: kernel tests, latency microbench (new vs one-wave panels).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k block_inverse --timeout 120 --timeout-method thread > gpurun_out/bi_test.log 2>&1
rc=$?; tail -15 gpurun_out/bi_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/bench_blockinv.py panel panel1 > gpurun_out/bi.log 2>&1 || exit $?
cat gpurun_out/bi.log
