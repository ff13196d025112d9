#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default twice.)
# MAIN updates the panel-after-next's columns first (GJ_STRIP) and/or the look-ahead rows on SIDE at
# p = 1 (GJ_LA_SIDE): same box, interleaved, two repetitions.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/strip
mkdir -p $o
for rep in 1 2; do
  for n in 8192 16384 32768; do
    st=10; [ $n = 32768 ] && st=3
    for v in "0 0" "1 0" "0 1" "1 1"; do
      set -- $v
      GJ_STRIP=$1 GJ_LA_SIDE=$2 timeout -k 10 200 python bench.py --size $n --steps $st --warmup 2 --no-residual > $o/n${n}_s$1_l$2_$rep.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/n${n}_s$1_l$2_$rep.json').read().splitlines()[-1]); print('n=$n strip=$1 la_side=$2 rep=$rep', d['ms_per_step'])"
    done
  done
done
