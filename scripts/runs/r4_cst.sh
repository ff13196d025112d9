#!/bin/bash
# COMM normalisation GEMMs on the 64 x 32 latency tile (GJ_COMM_SMALL_TILES) re-checked after the
# look-ahead rows moved to SIDE: N = 8192 (default on) and 16384 (default off).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/cst
mkdir -p $o
for rep in 1 2; do
  for v in "8192 1" "8192 0" "16384 0" "16384 1"; do
    set -- $v
    GJ_COMM_SMALL_TILES=$2 timeout -k 10 200 python bench.py --size $1 --steps 10 --warmup 2 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 small_tiles=$2', d['ms_per_step'], d['policy']['comm_small_tiles'])"
  done
done
