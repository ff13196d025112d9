#!/bin/bash
# Closing numbers on the final build: default bench (N = 32768 fp64), N = 8192 / 16384, fp32 N = 32768.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/close
mkdir -p $o
show() { python3 -c "import json; d=json.loads(open('$1').read().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d.get('check'), d.get('residual_ratio'))"; }
timeout -k 10 300 python bench.py > $o/default.json 2>&1 || { tail -5 $o/default.json; exit 1; }
show $o/default.json "default (N=32768 fp64)"
cp $o/default.json $o/default_bench.json
for rep in 1 2; do
  timeout -k 10 200 python bench.py --size 8192 --steps 20 --warmup 5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  show $o/b.json "n=8192"
  timeout -k 10 200 python bench.py --size 16384 --steps 5 --warmup 2 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  show $o/b.json "n=16384"
done
timeout -k 10 300 python bench.py --dtype fp32 --steps 3 --warmup 1 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
show $o/b.json "fp32 n=32768"
