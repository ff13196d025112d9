#!/bin/bash
# fp32 LDS-DMA 32x32x2 GEMM (GJ_GLDS32=<cfg>, -1 = the register-staged squarepf tile) vs the old path
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for c in 0 1 2 3 4; do
  GJ_GLDS32=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "dtype1 and (glds or auto or gemm_acc or store_identity)" --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || { tail -30 gpurun_out/f32_tests.log; exit 1; }
  echo "cfg=$c $(tail -1 gpurun_out/f32_tests.log)"
done
for c in -1 0 1 2 3 4; do
  for shape in "32768 16384 512" "16384 65536 512" "4096 65536 1024"; do
    GJ_GLDS32=$c timeout -k 10 60 python bench/gemm_probe.py $shape --dtype fp32 --variant auto --check 2>&1 | grep -v amdgpu.ids | sed "s/^/cfg=$c /" || exit 1
  done
done
for c in -1 0; do
  GJ_GLDS32=$c timeout -k 10 200 python bench.py --size 32768 --dtype fp32 --steps 3 > gpurun_out/f32.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['residual_inf'])" gpurun_out/f32.json "cfg=$c n=32768" || exit 1
done
