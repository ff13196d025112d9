#!/bin/bash
# Chunk-pass skip only under a CU reservation: N = 32768 (MAIN skip on/off, chunk pass split) and
# N = 8192 (both merged by default).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/skip2
mkdir -p $o
run() {  # size steps warmup skip
  GJ_SKIP_COLS=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 skip=$4', d['ms_per_step'])"
}
for rep in 1 2 3; do for k in 0 1; do run 32768 3 1 $k || exit 1; done; done
for rep in 1 2; do for k in 0 1; do run 8192 20 5 $k || exit 1; done; done
