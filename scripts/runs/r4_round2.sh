#!/bin/bash
# Second round-4 GPU session: the tests that failed in the first, the N = 8192 kernel trace, the
# same-box A/B against round 3 with the residency builds, and the GEMM stall counters.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py "tests/test_gpu_kernels.py::test_block_inverse_live_grid_matches_full_grid" -q --timeout 300 --timeout-method thread > gpurun_out/gputests2.txt 2>&1
rc=$?; tail -3 gpurun_out/gputests2.txt; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_profile.sh r4_8192 --size 8192 --steps 5 --warmup 2 --no-residual || exit $?
bash scripts/runs/r4_ab.sh
