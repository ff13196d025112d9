#!/bin/bash
# Early MAIN launch of the panel-after-next columns (GJ_EARLY_LA) A/B.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/early
mkdir -p $o
run() {  # size steps warmup e
  GJ_EARLY_LA=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 early=$4', d['ms_per_step'])"
}
for rep in 1 2; do for e in 0 1; do run 8192 20 5 $e || exit 1; done; done
for rep in 1 2; do for e in 0 1; do run 16384 5 2 $e || exit 1; done; done
for rep in 1 2; do for e in 0 1; do run 32768 3 1 $e || exit 1; done; done
for e in 0 1; do
  GJ_EARLY_LA=$e timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k early=$e"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
  GJ_EARLY_LA=$e timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu32k early=$e"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
