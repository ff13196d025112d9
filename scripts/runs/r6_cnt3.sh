#!/bin/bash
# Round 6: the non-temporal C tile re-checked on another box with the clock / power sampled (the
# closing box ran N = 32768 at 2364 MHz and 1313 W, below the power limit).  Driver command,
# alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/cnt3
mkdir -p $out
for rep in 1 2; do
  for c in 3 0; do
    GJ_MAIN_CNT=$c timeout -k 10 200 python3 scripts/smi_sample.py $out/smi_c${c}_$rep.jsonl -- python3 bench.py > $out/c${c}_$rep.json 2> $out/c${c}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/c${c}_$rep.json').read().strip().splitlines()[-1]); print('main_cnt $c', $rep, d['ms_per_step'], d['check'])"
    python3 scripts/smi_summary.py $out/smi_c${c}_$rep.jsonl | tail -1
  done
done
