#!/bin/bash
# Round 6: XCD tile-row groups of the trailing update (GJ_GLDS_GROUP 2 / 4 / 8) re-measured with the
# non-temporal C tile (more L2 left to the A slabs and the B band a group shares).  N = 32768,
# driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/groupnt
mkdir -p $out
for rep in 1 2; do
  for g in 4 8 2; do
    GJ_GLDS_GROUP=$g timeout -k 10 300 python3 bench.py > $out/g${g}_$rep.json 2> $out/g${g}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/g${g}_$rep.json').read().strip().splitlines()[-1]); print('group $g', $rep, d['ms_per_step'], d['check'])"
  done
done
