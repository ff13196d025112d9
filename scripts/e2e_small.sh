#!/bin/bash
# End-to-end check at the pivot-chain-bound sizes: bench.py at N=8192/16384 and the p-rank
# emulation at N=16384 (p = 4, 8) and N=32768 (p = 8).  BI=<variant> selects the block inverse.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for s in 8192 16384; do
  timeout -k 10 200 python bench.py --size $s --steps 5 > gpurun_out/e2e_$s.json 2>gpurun_out/e2e_$s.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/e2e_$s.json || exit 1
done
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 > gpurun_out/e2e_emu16k.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/e2e_emu16k.log
timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 > gpurun_out/e2e_emu32k.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/e2e_emu32k.log
