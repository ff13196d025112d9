#!/bin/bash
# Closing numbers after the register-fed latency kernel: N = 8192 / 16384 / 32768, the emulation
# table, the N = 8192 trace.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/final5b
mkdir -p $o
show() { python3 -c "import json; d=json.loads(open('$1').read().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d.get('check'), d.get('residual_ratio'))"; }
timeout -k 10 300 python bench.py > $o/default.json 2>&1 || { tail -5 $o/default.json; exit 1; }
show $o/default.json "default (N=32768 fp64)"
for rep in 1 2; do
  timeout -k 10 200 python bench.py --size 8192 --steps 20 --warmup 5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  show $o/b.json "n=8192"
  timeout -k 10 200 python bench.py --size 16384 --steps 5 --warmup 2 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  show $o/b.json "n=16384"
done
timeout -k 10 600 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --depth 0 --bw 50 100 --bcast both --reps 1 > $o/emu32k.txt 2>&1 || { tail -5 $o/emu32k.txt; exit 1; }
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 100 --bcast both --reps 1 > $o/emu16k.txt 2>&1 || { tail -5 $o/emu16k.txt; exit 1; }
cat $o/emu32k.txt $o/emu16k.txt | grep -h '"p"' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d['n'], d.get('depth'), d.get('bcast', 'free'), d.get('model_bw_gbs', ''), d['seconds'], d.get('comm_hidden', ''))"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof8k -o run -- python3 bench.py --size 8192 --steps 5 --warmup 2 --no-residual > $o/prof8k.log 2>&1 || { tail -5 $o/prof8k.log; exit 1; }
echo trace done
