#!/bin/bash
# Round-5 defaults (peeled 3-stage LDS-DMA trailing update; split off) on one box: GEMM kernel tests,
# then the one-GPU sizes against the round-4 kernel (GJ_GLDS_PEEL=0 GJ_GLDS_BUILD=2.3) interleaved,
# then the rank-0 emulation of p = 2 / 4 / 8 (MODEL of the interconnect, direct 50 GB/s).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/def5
mkdir -p $o
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -q -k "peeled or glds or deep_auto or elimination_extras or row_blocks" --timeout 120 --timeout-method thread > $o/tests.txt 2>&1
rc=$?; tail -2 $o/tests.txt; [ $rc -eq 0 ] || exit $rc
run() {
  local label=$1; shift
  env "$@" > $o/b.json 2> $o/b.err || { echo "$label FAILED"; tail -5 $o/b.err; return 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('$label', d['ms_per_step'], d.get('check'))"
}
for rep in 1 2; do
  run "n=32768 new" timeout -k 10 200 python bench.py --steps 3 --warmup 1 || exit 1
  run "n=32768 r4-kernel" GJ_GLDS_PEEL=0 GJ_GLDS_BUILD=2.3 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual || exit 1
done
for n in 16384 8192; do
  for rep in 1 2; do
    run "n=$n new" timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 || exit 1
    run "n=$n r4-kernel" GJ_GLDS_PEEL=0 timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 --no-residual || exit 1
  done
done
timeout -k 10 400 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu32k.txt 2>&1 || exit $?
grep -h '"p"' $o/emu32k.txt | cut -c1-260
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 2 > $o/emu16k.txt 2>&1 || exit $?
grep -h '"p"' $o/emu16k.txt | cut -c1-260
