#!/bin/bash
# GEMM tile-variant sweep at the trailing-update shape (each probe checks one call against torch fp64).
#   VARIANTS="narrow bigpf" SHAPE="32768 4096 512" DTYPES="fp64" bash scripts/gemm_variants.sh
cd "$(dirname "$0")/.." || exit 1
for v in ${VARIANTS:-narrow big bigpf squarepf glds}; do
  for dt in ${DTYPES:-fp64 fp32}; do
    timeout -k 10 60 python bench/gemm_probe.py ${SHAPE:-32768 4096 512} --variant $v --dtype $dt --check || exit $?
  done
done
