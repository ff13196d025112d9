#!/bin/bash
# Pivot-SIMD layout in the L2-image kernel (128 < m <= 256 fp64): kernel tests, batch latency.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "block_inverse" --timeout 200 --timeout-method thread > gpurun_out/bil2_test.log 2>&1 || { tail -30 gpurun_out/bil2_test.log; exit 1; }
tail -1 gpurun_out/bil2_test.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q -x -k "single_gpu_vs_numpy" --timeout 200 --timeout-method thread > gpurun_out/bil2_eng.log 2>&1 || { tail -30 gpurun_out/bil2_eng.log; exit 1; }
tail -1 gpurun_out/bil2_eng.log
for lay in 0 1 0 1; do
  GJ_BI_LAYOUT=$lay BI_M="192 256" BI_NBLK="64" timeout -k 10 120 python -u bench/bench_blockinv.py panel > gpurun_out/bil2_bench.log 2>&1 || { cat gpurun_out/bil2_bench.log; exit 1; }
  grep float64 gpurun_out/bil2_bench.log | sed "s/^/lay=$lay /"
done
