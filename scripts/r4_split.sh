#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default twice.)
# Co-resident candidate inverse with the fused selection: correctness (GPU engine tests with the
# co-resident form forced, and with the per-step split), then N = 8192 / 16384 with GJ_BI_SPLIT=0/1
# and the p = 2 / 4 ranks of N = 32768 (co-resident by default, now fused).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/split
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread > $o/kern.txt 2>&1
rc=$?; tail -1 $o/kern.txt; [ $rc -eq 0 ] || exit $rc
GJ_BI_CORESIDENT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 120 --timeout-method thread > $o/eng_co.txt 2>&1
rc=$?; tail -1 $o/eng_co.txt; [ $rc -eq 0 ] || exit $rc
GJ_BI_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 120 --timeout-method thread > $o/eng_split.txt 2>&1
rc=$?; tail -1 $o/eng_split.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for n in 8192 16384; do
    for sp in 0 1; do
      GJ_BI_SPLIT=$sp timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$n split=$sp', d['ms_per_step'], d['check'])"
    done
  done
done
timeout -k 10 600 python bench/bench_emulate.py --ranks 2 4 --size 32768 --reps 1 --bw 50 --bcast direct > $o/emu.txt 2>&1 || exit $?
grep '"seconds"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('emu', d['p'], d['n'], d.get('bcast', 'free'), d['seconds'])"
