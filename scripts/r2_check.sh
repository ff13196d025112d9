#!/bin/bash
# One-GPU state check: GPU test tier, bench.py at the BASELINE sizes, p-rank emulation.
# Every GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
for s in ${SIZES:-8192 16384 32768}; do
  timeout -k 10 200 python bench.py --size $s --steps ${STEPS:-5} > gpurun_out/bench_$s.json 2>gpurun_out/bench_$s.err || { tail -5 gpurun_out/bench_$s.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/bench_$s.json || exit 1
done
[ -n "$NO_EMU" ] && exit 0
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 16384 > gpurun_out/emu16k.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/emu16k.log
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 > gpurun_out/emu32k.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/emu32k.log
