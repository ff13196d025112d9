#!/bin/bash
# Block size 256 at N = 32768 on the round-4 build (live-candidate launches, host-free chain):
# K = 1024 trailing updates at depth 4 (512 at depth 2) against m = 128 / depth 4.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/m256
mkdir -p $o
for rep in 1 2; do
  for v in "128 4" "256 2" "256 4" "256 3"; do
    set -- $v
    timeout -k 10 300 python bench.py --block $1 --depth $2 --steps 3 --warmup 1 > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('m=$1 depth=$2', d['ms_per_step'], d['residual_inf'], d['check'], d['policy']['block_inverse'])"
  done
done
