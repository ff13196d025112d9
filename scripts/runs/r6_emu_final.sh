#!/bin/bash
# Round 6, closing: emulated rank 0 of p = 2 / 4 / 8 at N = 32768 and p = 4 / 8 at N = 16384 under
# the communication-cost model (direct 50 GB/s and 100 GB/s), final build.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/emufin
mkdir -p $out
timeout -k 10 400 python3 bench/bench_emulate.py --ranks 2 4 8 --size 32768 --bw 50 100 --bcast direct --reps 2 \
    > $out/emu32k.jsonl 2> $out/emu32k.err || { tail -5 $out/emu32k.err; exit 1; }
cut -c1-240 $out/emu32k.jsonl
timeout -k 10 300 python3 bench/bench_emulate.py --ranks 4 8 --size 16384 --bw 50 100 --bcast direct --reps 2 \
    > $out/emu16k.jsonl 2> $out/emu16k.err || { tail -5 $out/emu16k.err; exit 1; }
cut -c1-240 $out/emu16k.jsonl
