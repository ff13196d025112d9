#!/bin/bash
# Round-5 starting point on one box: N = 8192 / 16384 / 32768 timings of the round-4 build.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/r5base
mkdir -p $o
for v in "8192 20" "16384 10" "32768 5"; do
  set -- $v
  timeout -k 10 300 python bench.py --size $1 --steps $2 --warmup 2 > $o/b$1.json 2> $o/b$1.err || exit $?
  python3 -c "import json; d=json.loads(open('$o/b$1.json').read().splitlines()[-1]); print('n=$1', d['ms_per_step'], d.get('check'), d.get('residual'))"
done
