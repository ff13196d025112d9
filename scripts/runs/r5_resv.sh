#!/bin/bash
# CU reservation x depth re-check with the round-5 chain (host-free, live candidates, look-ahead rows
# on SIDE, LDS-DMA column updates) and the peeled trailing update.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/resv
mkdir -p $o
run() {  # size steps warmup reserve depth
  GJ_RESERVE_CUS=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --depth $5 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 reserve=$4 depth=$5', d['ms_per_step'])"
}
for rep in 1 2; do
  for cfg in "32 4" "0 4" "32 3" "0 3" "0 8" "32 8"; do run 16384 5 2 $cfg || exit 1; done
done
for rep in 1 2; do
  for cfg in "32 2" "0 2" "32 3" "0 3"; do run 8192 20 5 $cfg || exit 1; done
done
for cfg in "0 4" "32 4"; do run 20480 3 1 $cfg || exit 1; done
for cfg in "0 4" "32 4"; do run 24576 3 1 $cfg || exit 1; done
