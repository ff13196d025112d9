#!/bin/bash
# Panel-blocked candidate inverse for m > 256 (default) against the per-step global sweep
# (GJ variant "generic"): kernel tests, pivot rule, microbenchmark, and the engine at m = 512.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
[ -n "$SKIP_T" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "block_inverse" --timeout 200 --timeout-method thread > gpurun_out/bib_test.log 2>&1 || { tail -30 gpurun_out/bib_test.log; exit 1; }
tail -1 gpurun_out/bib_test.log
BI_M="300 512 1000" BI_NBLK="64" timeout -k 10 300 python -u bench/bench_blockinv.py ${BIV:-panel generic} > gpurun_out/bib_bench.log 2>&1 || { cat gpurun_out/bib_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bib_bench.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -q -x -k "single_gpu_vs_numpy and 1536" --timeout 150 --timeout-method thread > gpurun_out/bib_eng.log 2>&1 || { tail -20 gpurun_out/bib_eng.log; exit 1; }
tail -1 gpurun_out/bib_eng.log
for mm in ${MMS:-512 384}; do
  timeout -k 10 300 python bench.py --size 16384 --block $mm --steps 2 > gpurun_out/bib_b.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('m', d['config']['m'], 'depth', d['config']['depth'], d['ms_per_step'], 'ms', d['residual_inf'])" gpurun_out/bib_b.json || exit 1
done
