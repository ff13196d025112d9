#!/bin/bash
# Fused generate + norm (Device::generate_norm) vs generate then row_abs_max.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/gennorm
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "generated_norm" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {  # size steps warmup flag
  GJ_GEN_NORM=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 gen_norm=$4', d['ms_per_step'], d.get('check'))"
}
for rep in 1 2 3; do for k in 0 1; do run 32768 3 1 $k || exit 1; done; done
for k in 0 1; do run 8192 20 5 $k || exit 1; done
