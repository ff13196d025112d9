#!/bin/bash
# Power-of-two row strides in the fp64 trailing update: the solver's C is the X panel (row stride =
# the padded order, 256 KiB at N = 32768), A^T the multiplier panel (stride = local rows) and B a
# pivot-row chunk (stride = chunk width).  Same GEMM with each stride padded off the power of two.
set -o pipefail
cd "$(dirname "$0")/../.."
P="python bench/gemm_probe.py 32768 8192 512 --check"
for rep in 1 2; do
  for ld in "--ldc 8192" "--ldc 32768" "--ldc 32832" "--ldc 32784" "--ldc 32896" \
            "--ldc 32768 --lda 32832" "--ldc 32768 --ldb 8256" "--ldc 32832 --lda 32832 --ldb 8256"; do
    timeout -k 10 120 $P $ld || exit $?
  done
  timeout -k 10 120 python bench/gemm_probe.py 8192 4096 256 --ldc 8192 || exit $?
  timeout -k 10 120 python bench/gemm_probe.py 8192 4096 256 --ldc 8256 || exit $?
  timeout -k 10 120 python bench/gemm_probe.py 8192 4096 256 --ldc 8256 --lda 8256 --ldb 4160 || exit $?
  timeout -k 10 120 python bench/gemm_probe.py 4096 8192 1024 --ldc 32768 || exit $?
  timeout -k 10 120 python bench/gemm_probe.py 4096 8192 1024 --ldc 32832 --lda 4160 || exit $?
done
