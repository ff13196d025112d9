#!/bin/bash
# Average shader clock of the fp64 trailing-update GEMM, C += A B against C = A B: GRBM_GUI_ACTIVE
# (GPU-busy cycles) over the kernel's duration, one counter pass per run.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for op in acc store; do
  out=gpurun_out/clk_$op
  mkdir -p $out
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $out -o run -- \
      python3 bench/gemm_probe.py 32768 8192 512 --op $op --reps 10 > $out/probe.log 2>&1 || exit $?
  tail -1 $out/probe.log
done
