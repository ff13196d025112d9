#!/bin/bash
# Small-N follow-up after the look-ahead rows moved to SIDE: depth sweep at N = 8192 / 16384, then
# a kernel trace of N = 8192.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/small
mkdir -p $o
for n in 8192 16384; do
  for d in 2 3 4; do
    timeout -k 10 200 python bench.py --size $n --depth $d --steps 10 --warmup 2 --no-residual > $o/n${n}_d$d.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/n${n}_d$d.json').read().splitlines()[-1]); print('n=$n depth=$d', d['ms_per_step'])"
  done
done
bash scripts/gpu_profile.sh r4b_8192 --size 8192 --steps 5 --warmup 2 --no-residual
