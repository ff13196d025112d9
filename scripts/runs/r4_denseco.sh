#!/bin/bash
# N = 32768, one GPU: the 5-per-CU trailing update together with the co-resident inverse (which
# fits beside 3 trailing-update workgroups), depth 4 / 8, against the default; two repetitions.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/denseco
mkdir -p $o
for rep in 1 2; do
  for v in "4 0 0" "4 1 1" "8 1 1" "4 1 0"; do
    set -- $v
    GJ_DENSE_GEMM=$2 GJ_BI_CORESIDENT=$3 timeout -k 10 200 python bench.py --depth $1 --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('depth=$1 dense=$2 co=$3', d['ms_per_step'], d['policy']['block_inverse'], d['policy']['dense_gemm'])"
  done
done
