#!/bin/bash
# Pivot-chain wave priority A/B (GJ_CHAIN_PRIO: s_setprio of the chain's GEMM / owner-edit waves).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/cprio
mkdir -p $o
run() {  # size steps warmup prio
  GJ_CHAIN_PRIO=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 chain_prio=$4', d['ms_per_step'])"
}
for rep in 1 2; do for pr in 0 2 3; do run 8192 20 5 $pr || exit 1; done; done
for rep in 1 2; do for pr in 0 2; do run 16384 5 2 $pr || exit 1; done; done
for rep in 1 2; do for pr in 0 2; do run 32768 3 1 $pr || exit 1; done; done
for pr in 0 2; do
  GJ_CHAIN_PRIO=$pr timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k chain_prio=$pr"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
  GJ_CHAIN_PRIO=$pr timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu32k chain_prio=$pr"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
GJ_CHAIN_PRIO=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof8k -o run -- python3 bench.py --size 8192 --steps 5 --warmup 2 --no-residual > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
python3 scripts/side_chain.py $o/prof8k/run_results.db > $o/side.md; head -16 $o/side.md
