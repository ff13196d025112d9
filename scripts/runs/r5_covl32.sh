#!/bin/bash
# C-load overlap in the fp32 LDS-DMA kernel.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/covl32
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or glds" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2; do for c in 0 1; do
  GJ_GLDS_COVL=$c timeout -k 10 200 python bench.py --dtype fp32 --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('fp32 n=32768 covl=$c', d['ms_per_step'])"
done; done
timeout -k 10 300 python bench.py --dtype fp32 --size 65536 --steps 2 --warmup 1 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('fp32 n=65536', d['ms_per_step'], d.get('check'), d.get('residual'))"
