#!/bin/bash
# Lazy pair updates (GJ_LAZY=1): GPU engine tests with it on, then bench.py / p-rank emulation A/B.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
GJ_LAZY=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 300 --timeout-method thread > gpurun_out/lazy_test.log 2>&1 || { tail -30 gpurun_out/lazy_test.log; exit 1; }
tail -1 gpurun_out/lazy_test.log
for v in 0 1 0 1; do
  for s in ${SIZES:-32768 16384}; do
    GJ_LAZY=$v timeout -k 10 200 python bench.py --size $s --steps 3 > gpurun_out/lazy_b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('lazy', sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms', d['residual_inf'])" gpurun_out/lazy_b.json $v || exit 1
  done
done
for v in 0 1; do
  GJ_LAZY=$v timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 --size 32768 --reps 2 --bw 100 > gpurun_out/lazy_e.log 2>&1 || { tail -5 gpurun_out/lazy_e.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/lazy_e.log | grep model_bw | sed "s/^/lazy=$v /" | cut -c1-150
done
