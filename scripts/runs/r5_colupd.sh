#!/bin/bash
# The p = 1 chain column update (rows x 128 x j 128): LDS-DMA kernel (GJ_LAT_GLDS=1, default under
# the reservation) vs the register-fed latency kernel (GJ_LAT_GLDS=0 with lat_reg on).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/colupd
mkdir -p $o
run() {  # size steps warmup g
  GJ_LAT_GLDS=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 lat_glds=$4', d['ms_per_step'])"
}
for rep in 1 2 3; do for k in 1 0; do run 8192 20 5 $k || exit 1; done; done
for rep in 1 2; do for k in 1 0; do run 16384 5 2 $k || exit 1; done; done
