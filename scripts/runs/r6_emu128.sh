#!/bin/bash
# Round 6: emulated p = 2 / 4 / 8 ranks of N = 32768 (rank 0 on one GPU, bench/bench_emulate.py):
# the 128 x 64 tile forced vs the per-launch default (128 x 128 on ranks without a reservation),
# comm-free and under the direct 50 GB/s model.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/emu128
mkdir -p $out
for t in 64 0; do
  GJ_GLDS_TILE=$t timeout -k 10 300 python3 bench/bench_emulate.py --ranks 2 4 8 --size 32768 --bw 50 \
      --bcast direct --reps 2 > $out/emu_t$t.jsonl 2> $out/emu_t$t.err || { tail -5 $out/emu_t$t.err; exit 1; }
  cat $out/emu_t$t.jsonl | cut -c1-300
done
