#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default twice.)
# Incremental panel-column updates (GJ_INCR=1: rank-m update of the later panel columns after every
# step, column t+1 on SIDE, the rest on AUX) against the per-step K = j*m column update.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/incr
mkdir -p $o
for rep in 1 2; do
  for n in 16384 8192 32768; do
    st=10; [ $n = 32768 ] && st=3
    for i in 0 1; do
      GJ_INCR=$i timeout -k 10 200 python bench.py --size $n --steps $st --warmup 2 > $o/n${n}_i${i}_$rep.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/n${n}_i${i}_$rep.json').read().splitlines()[-1]); print('n=$n incr=$i rep=$rep', d['ms_per_step'], d['residual_inf'], d['check'])"
    done
  done
done
for i in 0 1; do
  GJ_INCR=$i timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --reps 2 --bw 50 --bcast direct > $o/emu16k_i$i.txt 2>&1 || exit $?
  GJ_INCR=$i timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct > $o/emu32k_i$i.txt 2>&1 || exit $?
  echo "incr=$i"; grep '"seconds"' $o/emu16k_i$i.txt $o/emu32k_i$i.txt | python3 -c "
import sys, json
for l in sys.stdin:
    f, _, j = l.partition(':'); d = json.loads(j); print(' ', d['p'], d['n'], d.get('bcast', 'free'), d['seconds'])"
done
GJ_INCR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 120 --timeout-method thread > $o/gputests.txt 2>&1
rc=$?; tail -2 $o/gputests.txt; exit $rc
