#!/bin/bash
# A-direct 128x128 fp64 GEMM (GJ_GEMM_VARIANT=dtva) against the LDS-DMA 128x64 kernel: kernel tests,
# alone at the solver's shapes (PG = A slices in flight 1 / 2), then inside the solver.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/dtva_test.log 2>&1 || { tail -30 gpurun_out/dtva_test.log; exit 1; }
tail -1 gpurun_out/dtva_test.log
for shape in "32768 8192 512" "32768 4096 512" "4096 32768 1024" "16384 8192 512" "8192 4096 256"; do
  timeout -k 10 120 python bench/gemm_probe.py $shape --variant glds --check || exit 1
  GJ_DTVA_PG=1 timeout -k 10 120 python bench/gemm_probe.py $shape --variant dtva --check || exit 1
  GJ_DTVA_PG=2 timeout -k 10 120 python bench/gemm_probe.py $shape --variant dtva --check || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/dtva_probe.log
[ -n "$NO_SOLVE" ] && exit 0
for v in 0 1 0 1; do
  GJ_DEEP_DTVA=$v timeout -k 10 200 python bench.py --steps 3 > gpurun_out/dtva_bench_$v.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('dtva', sys.argv[2], d['ms_per_step'], 'ms', d['residual_inf'])" gpurun_out/dtva_bench_$v.json $v || exit 1
done
