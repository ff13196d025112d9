#!/bin/bash
# Permute-kernel test, then panel depth at N = 32768 with the peeled K-slab kernel (K = d m).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/d32k
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "permute" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2; do for d in 4 8 6; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --depth $d --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=32768 depth=$d', d['ms_per_step'])"
done; done
