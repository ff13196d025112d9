#!/bin/bash
# Co-resident block inverse (GJ_BI_VARIANT=co) vs the register kernel: kernel tests, isolated
# latency, bench.py at N = 8192 / 16384 / 32768 with 0 / 32 reserved CUs, p = 8 emulation (cost model).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q -k "block_inverse" --timeout 120 --timeout-method thread > gpurun_out/co_tests.log 2>&1 || { tail -20 gpurun_out/co_tests.log; exit 1; }
tail -1 gpurun_out/co_tests.log
BI_NBLK="32 64 256" timeout -k 10 200 python bench/bench_blockinv.py panel co 2>&1 | grep float64 || exit 1
for v in panel co; do
  for n in 8192 16384 32768; do
    for rc in 0 32; do
      [ $n = 32768 ] && [ $rc = 32 ] && continue
      GJ_BI_VARIANT=$v GJ_RESERVE_CUS=$rc timeout -k 10 200 python bench.py --size $n --steps 3 --no-residual > gpurun_out/co.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/co.json "bi=$v n=$n reserve=$rc" || exit 1
    done
  done
  for rc in 0 32; do
    GJ_BI_VARIANT=$v GJ_RESERVE_CUS=$rc timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 100 2>&1 | grep -v amdgpu.ids | sed "s/^/bi=$v reserve=$rc /" || exit 1
    GJ_BI_VARIANT=$v GJ_RESERVE_CUS=$rc timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 --bw 100 2>&1 | grep -v amdgpu.ids | sed "s/^/bi=$v reserve=$rc /" || exit 1
  done
done
