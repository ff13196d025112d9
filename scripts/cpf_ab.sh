#!/bin/bash
# Next-tile C prefetch in the LDS-DMA GEMM (GJ_CPF = slices before the end, GJ_CPF_AHEAD = dispatch
# distance): alone at the solver's shapes, then in the solver.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
GJ_CPF=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/cpf_test.log 2>&1 || { tail -30 gpurun_out/cpf_test.log; exit 1; }
tail -1 gpurun_out/cpf_test.log
for shape in "32768 8192 512" "4096 32768 1024"; do
  for c in 0 2 4 8 16 0; do
    GJ_CPF=$c timeout -k 10 60 python bench/gemm_probe.py $shape --variant glds $([ $c = 4 ] && echo --check) | sed "s/^/cpf=$c /" || exit 1
  done
  for a in 768 1280; do
    GJ_CPF=4 GJ_CPF_AHEAD=$a timeout -k 10 60 python bench/gemm_probe.py $shape --variant glds | sed "s/^/cpf=4 ahead=$a /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cpf_probe.log
[ -n "$NO_SOLVE" ] && exit 0
for c in 0 ${CPF:-4} 0 ${CPF:-4}; do
  GJ_CPF=$c timeout -k 10 200 python bench.py --steps 3 > gpurun_out/cpf_bench.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('cpf', sys.argv[2], d['ms_per_step'], 'ms', d['residual_inf'])" gpurun_out/cpf_bench.json $c || exit 1
done
