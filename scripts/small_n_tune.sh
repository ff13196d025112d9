#!/bin/bash
# Pivot-chain-bound sizes after the matrix-core block inverse: depth x CU reservation x
# LDS-DMA GEMM from K=256 (GJ_GLDS_MINK), bench.py 3 timed inversions each.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in ${SIZES:-8192 16384}; do
  for d in 2 3 4; do
    for rc in 0 32 64; do
      for mk in 256 384; do
        GJ_RESERVE_CUS=$rc GJ_GLDS_MINK=$mk timeout -k 10 120 python bench.py --size $n --depth $d --steps 3 --no-residual > gpurun_out/tune.json 2>/dev/null || exit 1
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/tune.json "n=$n depth=$d reserve=$rc glds_mink=$mk" || exit 1
      done
    done
  done
done
