#!/bin/bash
# (1) deeper pipelines of the peeled trailing update (4 stages / 16-deep slices, both 3 per CU) vs the
# 3.3 default; (2) the RCCL channel footprint of a p = 2 solve; (3) the rank-0 emulation table with
# the measured footprint in the cost model (MODEL of the interconnect, not a measurement).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/next5
mkdir -p $o
for b in 3.3 4.3 16.2.3; do
  GJ_GLDS_BUILD=$b timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --ldc 32768 --reps 30 > $o/g.json 2>&1 || exit $?
  echo "gemm alone build=$b $(tail -1 $o/g.json | cut -c150-220)"
done
for rep in 1 2; do
  for b in 3.3 4.3 16.2.3; do
    GJ_GLDS_BUILD=$b timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=32768 build=$b', d['ms_per_step'])"
  done
done
bash scripts/runs/r5_rcclfp.sh || exit $?
timeout -k 10 500 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --depth 0 --bw 50 100 --bcast both --reps 1 > $o/emu32k.txt 2>&1 || exit $?
grep -h '"p"' $o/emu32k.txt | cut -c1-240
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 100 --bcast both --reps 1 > $o/emu16k.txt 2>&1 || exit $?
grep -h '"p"' $o/emu16k.txt | cut -c1-240
