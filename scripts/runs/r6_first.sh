#!/bin/bash
# Round 6: a shallower first panel (GJ_FIRST_DEPTH): MAIN idles until panel 0's pivot chain and its
# chunk pass are done (~0.45 ms at N = 8192, ~1.4 ms at N = 32768 after the generation); with one
# or two steps in panel 0 its first update starts earlier.  GPU kernel tests of the engine first,
# then driver-shaped runs, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/first
mkdir -p $out
GJ_FIRST_DEPTH=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py > $out/eng.log 2>&1
rc=$?; tail -2 $out/eng.log; [ $rc -eq 0 ] || exit $rc
run() {  # name size env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --size $n > $out/$name.json 2> $out/$name.err || return $?
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); p=d['policy']; print('$name', d['ms_per_step'], d['check'], d['residual_ratio'], p['depth'], p['first_depth'], p['nchunks'])"
}
for rep in 1 2; do
  run n8192_def_$rep 8192 GJ_NONE=0 || exit $?
  run n8192_f1_$rep 8192 GJ_FIRST_DEPTH=1 || exit $?
  run n16384_def_$rep 16384 GJ_NONE=0 || exit $?
  run n16384_f1_$rep 16384 GJ_FIRST_DEPTH=1 || exit $?
  run n16384_f2_$rep 16384 GJ_FIRST_DEPTH=2 || exit $?
  run n32768_def_$rep 32768 GJ_NONE=0 || exit $?
  run n32768_f1_$rep 32768 GJ_FIRST_DEPTH=1 || exit $?
  run n32768_f2_$rep 32768 GJ_FIRST_DEPTH=2 || exit $?
done
