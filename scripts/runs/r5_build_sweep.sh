#!/bin/bash
# Peeled-loop build per size: 2.5 (2 stages, 5 per CU) vs 3.3 (3 stages, 4 per CU), one box,
# interleaved, two repetitions (defaults: 2.5 under a CU reservation, i.e. N <= 16384; else 3.3).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/bsweep
mkdir -p $o
for rep in 1 2; do
  for v in "8192 20 2.5" "8192 20 3.3" "16384 10 2.5" "16384 10 3.3" "32768 3 3.3" "32768 3 2.5"; do
    set -- $v
    GJ_GLDS_BUILD=$3 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 build=$3', d['ms_per_step'])"
  done
done
