#!/bin/bash
# N = 32768, one GPU: register candidate inverse vs the co-resident one (selection now fused into
# it), at depth 4 and 8; interleaved, two repetitions.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/cofused
mkdir -p $o
for rep in 1 2; do
  for v in "4 0" "4 1" "8 1" "8 0"; do
    set -- $v
    GJ_BI_CORESIDENT=$2 timeout -k 10 200 python bench.py --depth $1 --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('depth=$1 co=$2', d['ms_per_step'], d['policy']['block_inverse'])"
  done
done
