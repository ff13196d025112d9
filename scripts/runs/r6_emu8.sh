#!/bin/bash
# Round 6: emulated p = 8 ranks of N = 32768 (4096 rows, 32 CUs reserved, depth 8): the trailing
# update's build / tile (5-per-CU 128 x 64 default, 4-per-CU 128 x 64, 3-per-CU 128 x 128).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/emu8
mkdir -p $out
for cfg in "def GJ_NONE=0" "nodense GJ_DENSE_GEMM=0" "t128 GJ_DENSE_GEMM=0 GJ_GLDS_TILE=128"; do
  set -- $cfg
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench/bench_emulate.py --ranks 8 --size 32768 --bw 50 --bcast direct --reps 2 \
      > $out/$name.jsonl 2> $out/$name.err || { tail -5 $out/$name.err; exit 1; }
  echo $name; cut -c1-220 $out/$name.jsonl
done
