#!/bin/bash
# Round 6: emulated ranks of p = 2 / 4 at N = 32768 (16384- / 8192-row ranks, no reservation):
# the co-resident candidate inverse (their auto choice) against the register form, on the round-6
# trailing-update tiles.  Comm-free and direct 50 GB/s.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/emuco
mkdir -p $out
for rep in 1 2; do
  for co in 1 0; do
    GJ_BI_CORESIDENT=$co timeout -k 10 400 python3 bench/bench_emulate.py --ranks 2 4 --size 32768 --bw 50 --bcast direct --reps 2 \
        > $out/co${co}_$rep.jsonl 2> $out/co${co}_$rep.err || { tail -5 $out/co${co}_$rep.err; exit 1; }
    echo "coresident $co rep $rep"; cut -c1-200 $out/co${co}_$rep.jsonl
  done
done
