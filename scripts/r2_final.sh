#!/bin/bash
# Round-2 state on one GPU: GPU tests, bench.py at the BASELINE sizes, p-rank emulation with the
# engine's own choices (comm-free + 100 GB/s cost model), rocprofv3 trace of the headline.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_final.log 2>&1 || { tail -30 gpurun_out/gt_final.log; exit 1; }
tail -1 gpurun_out/gt_final.log
for s in 8192 16384 32768; do
  timeout -k 10 200 python bench.py --size $s --steps 5 > gpurun_out/final_$s.json 2>gpurun_out/final_$s.err || { tail -5 gpurun_out/final_$s.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/final_$s.json || exit 1
done
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --reps 2 --bw 50 100 > gpurun_out/final_emu.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/final_emu.log
out=gpurun_out/prof_final_32768
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 bench.py --size 32768 --steps 1 --warmup 1 --no-residual > $out/bench.log 2>&1 || exit 1
db=$(find $out -name "*.db" | head -1)
python3 scripts/rocpd_summary.py "$db" > $out/summary.md && head -22 $out/summary.md
