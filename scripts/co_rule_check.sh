#!/bin/bash
# Engine rule: co-resident candidate inverse on p > 1 ranks without a CU reservation.  GPU engine
# tests, then the p = 2 / 4 / 8 emulation (default rule vs forced off) and the 1-GPU headline.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 300 --timeout-method thread > gpurun_out/co_rule_test.log 2>&1 || { tail -30 gpurun_out/co_rule_test.log; exit 1; }
tail -1 gpurun_out/co_rule_test.log
for v in 1 0 1 0; do
  GJ_BI_CORESIDENT=$v timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --reps 2 --bw 100 > gpurun_out/cr.log 2>&1 || { tail -5 gpurun_out/cr.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/cr.log | grep model_bw | sed "s/^/co=$v /" | cut -c1-150
done
timeout -k 10 200 python bench.py --steps 3 > gpurun_out/cr_b.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('p1', d['ms_per_step'], 'ms', d['residual_inf'])" gpurun_out/cr_b.json
