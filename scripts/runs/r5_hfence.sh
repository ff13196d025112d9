#!/bin/bash
# Host pivot mirror: system-scope relaxed stores (default) vs system-scope fences (GJ_HOST_FENCE=1).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/hfence
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {  # size steps warmup fence
  GJ_HOST_FENCE=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 fence=$4', d['ms_per_step'])"
}
for rep in 1 2; do for k in 1 0; do run 8192 20 5 $k || exit 1; done; done
for k in 1 0; do run 16384 5 2 $k || exit 1; done
for rep in 1 2; do for k in 1 0; do
  GJ_HOST_FENCE=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --bw 50 --bcast direct --reps 2 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k fence=$k"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done; done
for k in 1 0; do
  GJ_HOST_FENCE=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu32k fence=$k"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 > $o/emu.log 2>&1 || { tail -5 $o/emu.log; exit 1; }
python3 scripts/side_chain.py $o/prof/run_results.db 128 2 > $o/side.md; cat $o/side.md
