#!/bin/bash
# Chunk width sweep at N = 8192 / 16384 (trailing-update launch tails vs the chunk-pass pipeline).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/chunks
mkdir -p $o
run() {  # size steps warmup chunk
  timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --chunk-cols $4 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 chunk=$4', d['ms_per_step'], d['config'].get('policy', {}).get('nchunks'))"
}
for rep in 1 2; do for c in 4096 2048 2560 2816 3072 3584 5376 8192; do run 8192 20 5 $c || exit 1; done; done
for rep in 1 2; do for c in 8192 3584 4096 4608 5120 6144 7168 16384; do run 16384 5 2 $c || exit 1; done; done
