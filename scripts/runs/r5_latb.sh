#!/bin/bash
# The piece batch on the register-fed tile (GJ_LAT_BATCH) A/B, N = 8192 / 16384 and emulated p = 8.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/latb
mkdir -p $o
run() {  # size steps warmup k
  GJ_LAT_BATCH=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 lat_batch=$4', d['ms_per_step'])"
}
for rep in 1 2 3; do for k in 0 1; do run 8192 20 5 $k || exit 1; done; done
for rep in 1 2; do for k in 0 1; do run 16384 5 2 $k || exit 1; done; done
for k in 0 1 0 1; do
  GJ_LAT_BATCH=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  GJ_LAT_BATCH=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 >> $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu lat_batch=$k: $(grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
print(' '.join('%s/%s/%s=%s' % (d['p'], d['n'], d.get('bcast', 'free'), d['seconds']) for d in map(json.loads, sys.stdin)))")"
done
