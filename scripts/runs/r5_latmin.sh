#!/bin/bash
# Small pivot-chain GEMMs (m x q m x m pieces, look-ahead rows) on the LDS-DMA kernel too.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/latmin
mkdir -p $o
run() {  # size steps warmup min
  GJ_LAT_GLDS_MIN=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 lat_glds_min=$4', d['ms_per_step'])"
}
for rep in 1 2; do for k in 1024 128; do run 8192 20 5 $k || exit 1; done; done
for rep in 1 2; do for k in 1024 128; do run 16384 5 2 $k || exit 1; done; done
