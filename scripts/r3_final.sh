#!/bin/bash
# Round-3 closing measurements: K = 256 kernel choice, one-GPU sizes, rocprofv3 summary at N = 32768.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab.sh -r 2 -t 100 -v "auto:" -v "glds:GJ_GEMM_VARIANT=glds" -v "narrow:GJ_GEMM_VARIANT=narrow" -- \
    python bench/gemm_probe.py 8192 4096 256 && \
bash scripts/ab.sh -r 2 -t 200 -v "auto:" -v "glds:GJ_GEMM_VARIANT=glds" -- python bench.py --size 8192 --steps 5 --warmup 2 && \
bash scripts/ab.sh -r 2 -t 200 -v "auto:" -v "glds:GJ_GEMM_VARIANT=glds" -- python bench.py --size 16384 --steps 3 --warmup 1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 && \
mkdir -p gpurun_out/prof_r3 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-residual > gpurun_out/prof_r3/bench.log 2>&1
