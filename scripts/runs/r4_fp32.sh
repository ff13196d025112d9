#!/bin/bash
# BASELINE config 5: N = 65536 fp32 on one GPU (and N = 32768 fp32 for the table).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/fp32
mkdir -p $o
for n in 32768 65536; do
  timeout -k 10 400 python bench.py --size $n --dtype fp32 --steps 2 --warmup 1 > $o/b$n.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/b$n.json').read().splitlines()[-1]); print('fp32 n=$n', d['ms_per_step'], d['value'], d['residual_inf'], d['check'], d['policy'])"
done
