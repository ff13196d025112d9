#!/bin/bash
# Round 6: one MAIN launch around the look-ahead columns (GJ_SKIP_COLS=1) at N = 32768 with the
# 128 x 128 tile: its split chunks run 3072 + 12288 ... tiles in two launches, each with a tail of
# 3-per-CU 128 x 128 tiles (round 5 measured the merge +0.1-0.3 % with the 128 x 64 tile).  The
# chunk-pass merge stays off (GJ_CHUNK_SKIP=0; +1.5 % in round 5).  Driver command, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/skip128
mkdir -p $out
for rep in 1 2; do
  for cfg in def skip; do
    if [ $cfg = skip ]; then export GJ_SKIP_COLS=1 GJ_CHUNK_SKIP=0; else unset GJ_SKIP_COLS GJ_CHUNK_SKIP; fi
    timeout -k 10 300 python3 bench.py > $out/${cfg}_$rep.json 2> $out/${cfg}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/${cfg}_$rep.json').read().strip().splitlines()[-1]); print('$cfg', $rep, d['ms_per_step'], d['check'], d['residual_ratio'], d['policy']['skip_cols'])"
  done
done
