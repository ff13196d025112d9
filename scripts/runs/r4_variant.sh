#!/bin/bash
# Every non-latency GEMM launch on the LDS-DMA kernel (GJ_GEMM_VARIANT=glds: also the look-ahead
# update on SIDE and the COMM normalisation GEMMs, which the auto rule leaves on the register-staged
# 128 x 64 tile below 512 tiles) vs the auto rule.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/variant
mkdir -p $o
for rep in 1 2; do
  for v in auto glds; do
    for n in 8192 16384 32768; do
      st=10; [ $n = 32768 ] && st=3
      GJ_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --size $n --steps $st --warmup 2 > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('variant=$v n=$n', d['ms_per_step'], d['check'])"
    done
  done
done
