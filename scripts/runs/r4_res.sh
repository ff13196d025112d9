#!/bin/bash
# CU reservation 32 vs 64 at the chain-bound configurations, now that the reserved-CU trailing update
# runs 5 workgroups per CU (dense).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/res
mkdir -p $o
for rc in 32 64; do
  for n in 8192 16384; do
    GJ_RESERVE_CUS=$rc timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 --no-residual > $o/n${n}_r$rc.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/n${n}_r$rc.json').read().splitlines()[-1]); print('n=$n res=$rc', d['ms_per_step'])"
  done
  GJ_RESERVE_CUS=$rc timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --reps 2 --bw 50 --bcast direct > $o/emu16k_r$rc.txt 2>&1 || exit $?
  echo "res=$rc"; grep '"seconds"' $o/emu16k_r$rc.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['p'], d['n'], d.get('bcast', 'free'), d['seconds'])"
done
