#!/bin/bash
# COMM on MAIN's 224-CU mask (GJ_COMM_MASK=1) vs unmasked high-priority COMM (default).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/commmask
mkdir -p $o
run() {  # size steps warmup flag [extra]
  GJ_COMM_MASK=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 $5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 commmask=$4', d['ms_per_step'], d.get('check', ''))"
}
run 8192 10 3 1 || exit 1
for rep in 1 2; do for k in 0 1; do run 8192 20 5 $k --no-residual || exit 1; done; done
for rep in 1 2; do for k in 0 1; do run 16384 5 2 $k --no-residual || exit 1; done; done
for k in 0 1; do
  GJ_COMM_MASK=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --bw 50 --bcast direct --reps 2 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k commmask=$k"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
