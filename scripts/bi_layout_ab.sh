#!/bin/bash
# Matrix-core block inverse with the pivot wave alone on its SIMD (GJ_BI_LAYOUT=1: idle hardware
# waves 4, 8) vs the default 9-wave layout: kernel tests, batch latency, engine.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
GJ_BI_LAYOUT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "block_inverse" --timeout 200 --timeout-method thread > gpurun_out/bil_test.log 2>&1 || { tail -30 gpurun_out/bil_test.log; exit 1; }
tail -1 gpurun_out/bil_test.log
for lay in 0 1 0 1; do
  GJ_BI_LAYOUT=$lay BI_M="64 128" BI_NBLK="32 64 256" timeout -k 10 120 python -u bench/bench_blockinv.py panel > gpurun_out/bil_bench.log 2>&1 || { cat gpurun_out/bil_bench.log; exit 1; }
  grep float64 gpurun_out/bil_bench.log | sed "s/^/lay=$lay /"
done
for lay in 0 1 0 1; do
  for s in 8192 16384 32768; do
    GJ_BI_LAYOUT=$lay timeout -k 10 200 python bench.py --size $s --steps 3 --no-residual > gpurun_out/bil_b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('lay', sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms')" gpurun_out/bil_b.json $lay || exit 1
  done
done
