#!/bin/bash
# Round-3 closing measurements (one box): one-GPU sizes and the p-rank emulation table under the
# direct-broadcast cost model.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for n in 8192 16384; do
  timeout -k 10 200 python bench.py --size $n --steps 5 --warmup 2 || exit $?
done && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 && \
timeout -k 10 400 python bench/bench_emulate.py --ranks 2 4 8 --size 32768 --reps 1 --bw 50 --bcast direct && \
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 16384 --reps 1 --bw 50 --bcast direct
