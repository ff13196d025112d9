#!/bin/bash
# LDS-DMA GEMM sweep: pipeline stages x tile-row grouping at the trailing-update shape.
cd "$(dirname "$0")/.." || exit 1
for st in ${STAGES:-2 3 4 5}; do
  for gp in ${GRP_LIST:-1 4 8 16}; do
    echo -n "stages=$st group=$gp "
    GJ_GLDS_STAGES=$st GJ_GEMM_GROUP=$gp timeout -k 10 60 python bench/gemm_probe.py ${SHAPE:-32768 4096 512} --variant glds --check 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
