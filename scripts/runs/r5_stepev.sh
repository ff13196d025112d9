#!/bin/bash
# SIDE records ev_edit_ / ev_pp_ only after a panel's last step (default) vs every step (GJ_STEP_EVENTS=1).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/stepev
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_golden_residuals.py -m gpu > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {  # size steps warmup flag [extra]
  GJ_STEP_EVENTS=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 $5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 stepev=$4', d['ms_per_step'], d.get('check', ''))"
}
run 8192 10 3 0 || exit 1
for rep in 1 2 3; do for k in 1 0; do run 8192 20 5 $k --no-residual || exit 1; done; done
for rep in 1 2; do for k in 1 0; do run 16384 5 2 $k --no-residual || exit 1; done; done
for k in 1 0; do
  GJ_STEP_EVENTS=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --bw 50 --bcast direct --reps 2 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k stepev=$k"; grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['p'], d.get('bcast', 'free'), d['seconds'])"
done
