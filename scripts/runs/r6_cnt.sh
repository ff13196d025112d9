#!/bin/bash
# Round 6: the trailing update's C tile through the non-temporal cache policy (GJ_GLDS_CNT: bit 0
# loads, bit 1 stores).  Each C element is read and written once per panel and not again until the
# next panel's pass over 8.6 GB; streaming it might leave L2 / MALL to the A and B operands (less
# HBM traffic per flop under the power limit).  The new first-depth / chunk-plan GPU test first;
# then the driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/cnt
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py -k "first_depth" > $out/test.log 2>&1
rc=$?; tail -2 $out/test.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in 0 1 2 3; do
    GJ_GLDS_CNT=$c timeout -k 10 300 python3 bench.py > $out/c${c}_$rep.json 2> $out/c${c}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/c${c}_$rep.json').read().strip().splitlines()[-1]); print('cnt $c', $rep, d['ms_per_step'], d['check'], d['residual_ratio'])"
  done
done
