#!/bin/bash
# Round 6: column-chunk plans at N = 32768 (GJ_CHUNK_PLAN, block counts of 128 columns).  MAIN's
# 128 x 128 tiles, 3 per CU on 256 CUs = 768 per wave = 3 block columns per wave; a panel's update
# is 84 waves of tiles (the look-ahead's 4 block columns skipped), the auto plan (4 x 64 blocks)
# launches it as 20 + 3 x 21.33 waves.  Plans in multiples of 12 blocks end on whole waves.
# Driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/plan32k
mkdir -p $out
for rep in 1 2; do
  for plan in auto 60,60,72,64 84,84,88 48,48,48,48,64 96,96,64; do
    if [ $plan = auto ]; then unset GJ_CHUNK_PLAN; else export GJ_CHUNK_PLAN=$plan; fi
    timeout -k 10 300 python3 bench.py > $out/p${plan}_$rep.json 2> $out/p${plan}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/p${plan}_$rep.json').read().strip().splitlines()[-1]); print('$plan', $rep, d['ms_per_step'], d['check'], d['residual_ratio'])"
  done
done
