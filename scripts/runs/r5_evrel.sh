#!/bin/bash
# Ordering-event release scope: system (HIP default) vs device vs none (GJ_EVENT_RELEASE).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/evrel
mkdir -p $o
GJ_EVENT_RELEASE=device timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {  # size steps warmup mode [extra]
  GJ_EVENT_RELEASE=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 $5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 ev=$4', d['ms_per_step'], d.get('check', ''), d.get('residual_inf', ''))"
}
for k in system device none; do run 8192 10 3 $k || exit 1; done
for rep in 1 2; do for k in system device none; do run 8192 20 5 $k --no-residual || exit 1; done; done
for k in system device none; do run 16384 5 2 $k --no-residual || exit 1; done
for k in system device none; do
  GJ_EVENT_RELEASE=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --bw 50 --bcast direct --reps 2 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k ev=$k"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
GJ_EVENT_RELEASE=device timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 > $o/emu.log 2>&1 || { tail -5 $o/emu.log; exit 1; }
python3 scripts/side_chain.py $o/prof/run_results.db 128 2 > $o/side.md; cat $o/side.md
