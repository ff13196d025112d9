#!/bin/bash
# 128 x 128 LDS-DMA GEMM (GJ_GLDS_DEEP=12) vs the 128 x 64 one (11): correctness, alone, in the solver.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "glds" --timeout 120 --timeout-method thread > gpurun_out/glds128_tests.log 2>&1 || { tail -20 gpurun_out/glds128_tests.log; exit 1; }
tail -1 gpurun_out/glds128_tests.log
for shape in "32768 4096 512" "32768 8192 512" "4096 32768 1024" "16384 8192 512"; do
  for v in glds glds128; do
    timeout -k 10 60 python bench/gemm_probe.py $shape --variant $v --check 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for rep in 1 2; do
  for d in 11 12; do
    for n in 16384 32768; do
      GJ_GLDS_DEEP=$d timeout -k 10 200 python bench.py --size $n --steps 3 --no-residual > gpurun_out/g128.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/g128.json "deep=$d n=$n" || exit 1
    done
  done
done
for d in 11 12; do
  GJ_GLDS_DEEP=$d timeout -k 10 300 python bench/bench_emulate.py --ranks 2 8 --size 32768 --reps 2 --bw 100 2>&1 | grep -v amdgpu.ids | sed "s/^/deep=$d /" || exit 1
done
