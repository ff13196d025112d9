#!/bin/bash
# Round 6: the non-temporal C tile in the fp32 LDS-DMA kernel (MAIN's launches, the engine default)
# against none, N = 32768 fp32, driver-shaped runs, one box, alternating; bit-identity tests first.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/cnt32
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py -k "nontemporal" > $out/test.log 2>&1
rc=$?; tail -2 $out/test.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in 3 0; do
    GJ_MAIN_CNT=$c timeout -k 10 300 python3 bench.py --dtype fp32 > $out/c${c}_$rep.json 2> $out/c${c}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/c${c}_$rep.json').read().strip().splitlines()[-1]); print('fp32 main_cnt $c', $rep, d['ms_per_step'], d['check'])"
  done
done
