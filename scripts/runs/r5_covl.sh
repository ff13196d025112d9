#!/bin/bash
# C loads of the LDS-DMA trailing update overlapped with the first K slices (GJ_GLDS_COVL) vs before them.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/covl
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or glds" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2; do for c in 0 1; do
  GJ_GLDS_COVL=$c timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --ldc 32768 --reps 30 > $o/g.json 2>&1 || { tail -5 $o/g.json; exit 1; }
  echo "gemm alone covl=$c $(tail -1 $o/g.json | cut -c150-220)"
done; done
run() {  # size steps warmup c
  GJ_GLDS_COVL=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 covl=$4', d['ms_per_step'])"
}
for rep in 1 2 3; do for c in 0 1; do run 32768 3 1 $c || exit 1; done; done
for rep in 1 2; do for c in 0 1; do run 16384 5 2 $c || exit 1; done; done
for rep in 1 2; do for c in 0 1; do run 8192 20 5 $c || exit 1; done; done
