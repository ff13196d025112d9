#!/bin/bash
# Round 6: emulated p = 8 ranks of N = 32768: the 32-CU reservation against none (co-resident
# candidate inverse), comm-free and direct 50 GB/s.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/emu8res
mkdir -p $out
for r in 32 0; do
  GJ_RESERVE_CUS=$r timeout -k 10 300 python3 bench/bench_emulate.py --ranks 8 --size 32768 --bw 50 --bcast direct --reps 2 \
      > $out/r$r.jsonl 2> $out/r$r.err || { tail -5 $out/r$r.err; exit 1; }
  echo reserve $r; cut -c1-200 $out/r$r.jsonl
done
for d in 4 8; do
  GJ_RESERVE_CUS=0 timeout -k 10 300 python3 bench/bench_emulate.py --ranks 8 --size 32768 --depth $d --bw 50 --bcast direct --reps 2 \
      > $out/r0d$d.jsonl 2> $out/r0d$d.err || { tail -5 $out/r0d$d.err; exit 1; }
  echo reserve 0 depth $d; cut -c1-200 $out/r0d$d.jsonl
done
