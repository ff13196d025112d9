#!/bin/bash
# A/B of the peeled, stage-unrolled LDS-DMA trailing-update loop (GJ_GLDS_PEEL) against the general
# loop: numerics test, the GEMM alone at the solver's chunk shape, and the solve at three sizes,
# interleaved over two repetitions.  2.3 = 2 stages (default), 3.3 = 3 stages, both 4 per CU.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/peel
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "glds_peeled or deep_auto or elimination_extras" --timeout 120 --timeout-method thread > $o/tests.txt 2>&1
rc=$?; tail -3 $o/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for b in 2.3 3.3; do
    for p in 0 1; do
      GJ_GLDS_BUILD=$b GJ_GLDS_PEEL=$p timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --ldc 32768 --reps 30 > $o/g.json 2>&1 || exit $?
      echo "gemm build=$b peel=$p $(tail -1 $o/g.json)"
    done
  done
done
for rep in 1 2; do
  for b in 2.3 3.3; do
    for p in 0 1; do
      GJ_GLDS_BUILD=$b GJ_GLDS_PEEL=$p timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=32768 build=$b peel=$p', d['ms_per_step'])"
    done
  done
done
for rep in 1 2; do
  for n in 16384 8192; do
    for p in 0 1; do
      GJ_GLDS_PEEL=$p timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 --no-residual > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$n peel=$p', d['ms_per_step'])"
    done
  done
done
