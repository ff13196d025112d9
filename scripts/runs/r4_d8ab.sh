#!/bin/bash
# Same-box A/B at N = 32768: depth 4 + register inverse (round-4 start) vs the depth-8 +
# co-resident default, 5 timed steps each, interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/d8ab
mkdir -p $o
for rep in 1 2 3; do
  for v in a b; do
    if [ $v = a ]; then env="GJ_BI_CORESIDENT=0"; d=4; else env="GJ_BI_CORESIDENT=1"; d=8; fi
    env $env timeout -k 10 300 python bench.py --depth $d --steps 5 --warmup 2 --no-residual > $o/${v}_$rep.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/${v}_$rep.json').read().splitlines()[-1]); print('$v', $rep, d['ms_per_step'], d['policy']['depth'], d['policy']['block_inverse'])"
  done
done
