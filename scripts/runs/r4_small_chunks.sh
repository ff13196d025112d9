#!/bin/bash
# Chunk width at the chain-bound sizes: narrower trailing-update launches give the pivot chain's
# high-priority workgroups more launch boundaries to start at.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/schunk
mkdir -p $o
for rep in 1 2; do
  for v in "8192 4096" "8192 8192" "16384 8192" "16384 16384"; do
    set -- $v
    timeout -k 10 200 python bench.py --size $1 --chunk-cols $2 --steps 10 --warmup 2 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 chunk=$2', d['ms_per_step'], d['policy']['nchunks'])"
  done
done
