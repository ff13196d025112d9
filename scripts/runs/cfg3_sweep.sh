#!/bin/bash
# BASELINE config 3 neighbourhood: emulated p = 4 / 8 ranks of N = 16384 (direct 50 GB/s model),
# depth x chunk width.
set -o pipefail
cd "$(dirname "$0")/../.."
for cc in 0 4096 2048; do
  timeout -k 10 300 python bench/bench_emulate.py --ranks 4 --size 16384 --reps 1 --bw 50 --bcast direct \
      --depth 3 4 5 6 --chunk-cols $cc || exit $?
done
for cc in 0 4096; do
  timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 16384 --reps 1 --bw 50 --bcast direct \
      --depth 2 3 4 6 --chunk-cols $cc || exit $?
done
