#!/bin/bash
# p = 8 ranks of N = 32768 without the CU reservation, register candidate inverse (depth 8)
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/ab.sh -r 2 -t 200 -v "dflt:" -v "r0reg:GJ_RESERVE_CUS=0 GJ_BI_CORESIDENT=0" -- \
    python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct
