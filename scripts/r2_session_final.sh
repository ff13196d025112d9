#!/bin/bash
# End-of-session evidence on one GPU: the whole GPU test tier, bench.py at the BASELINE sizes
# (fp64 8192 / 16384 / 32768, fp32 65536), and a rocprofv3 kernel trace of the N = 32768 headline.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gt.log 2>&1 || { tail -30 gpurun_out/final_gt.log; exit 1; }
tail -1 gpurun_out/final_gt.log
for s in 8192 16384 32768; do
  timeout -k 10 300 python bench.py --size $s --steps 5 > gpurun_out/final_b_$s.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], d['dtype'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/final_b_$s.json || exit 1
done
timeout -k 10 300 python bench.py --size 65536 --dtype fp32 --steps 2 > gpurun_out/final_b_65536.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], d['dtype'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', round(d['value']/1e3,1), 'TF', d['residual_inf'])" gpurun_out/final_b_65536.json || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_final_r2s
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 bench.py --steps 1 --warmup 1 > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
db=$(find $out -name "*.db" | head -1)
python3 scripts/rocpd_summary.py "$db" > gpurun_out/final_prof_summary.md 2>&1 || exit 1
python3 scripts/main_gaps.py "$db" > gpurun_out/final_prof_gaps.txt 2>&1 || exit 1
head -12 gpurun_out/final_prof_summary.md
