#!/bin/bash
# Round 6: uneven column-chunk plans at N = 8192 (GJ_CHUNK_PLAN, block counts).  MAIN's chunk GEMM
# runs W / 64 x 64 tiles of 128 x 64 on 224 CUs x 4 slots = 896 per wave, i.e. 7 block columns per
# wave: 32 + 32 blocks take 5 + 5 waves for 8.9 waves of work; 28 + 36 / 34 + 30 take 9 for about
# half of the panels.  Driver-shaped 20/5 runs, two alternating repetitions.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/plan8k
mkdir -p $out
for rep in 1 2; do
  for plan in auto 28,36 36,28 34,30 30,34 64; do
    if [ $plan = auto ]; then unset GJ_CHUNK_PLAN; else export GJ_CHUNK_PLAN=$plan; fi
    timeout -k 10 200 python3 bench.py --size 8192 > $out/p${plan}_$rep.json 2> $out/p${plan}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/p${plan}_$rep.json').read().strip().splitlines()[-1]); print('$plan', $rep, d['ms_per_step'], d['check'], d['residual_ratio'])"
  done
done
