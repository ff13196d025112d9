#!/bin/bash
# Round 6: the 128 x 128 tile at the small BASELINE sizes (A/B, driver-shaped 20/5 runs), N = 16384
# with the 4-per-CU tile-128 build instead of the 5-per-CU dense one; the no-fence run without
# verification (does it still reproduce?).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/s128
mkdir -p $out
for rep in 1 2; do
  for cfg in "8192 64 auto" "8192 128 auto" "16384 64 auto" "16384 128 auto" "16384 128 0"; do
    set -- $cfg
    if [ $3 = auto ]; then de=""; else de="GJ_DENSE_GEMM=$3"; fi
    env GJ_GLDS_TILE=$2 $de timeout -k 10 120 python3 bench.py --size $1 > $out/b$1_$2_$3_$rep.json 2> $out/b$1_$2_$3_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/b$1_$2_$3_$rep.json').read().strip().splitlines()[-1]); print('$cfg', $rep, d['ms_per_step'], d['check'])"
  done
done
GJ_EVENT_RELEASE=none timeout -k 10 300 python3 scripts/runs/r6_nofence.py > $out/nofence_noverify.jsonl 2> $out/nofence_noverify.err || exit $?
cut -c1-200 $out/nofence_noverify.jsonl
