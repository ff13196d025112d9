#!/bin/bash
# Round 6: non-temporal C on MAIN's trailing update only (the engine default, GemmExtra::c_nt = 3)
# against none (GJ_MAIN_CNT=0) and against every LDS-DMA launch (GJ_GLDS_CNT=3), at the BASELINE
# sizes.  Bit-identity test first; driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/cnt2
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py -k "nontemporal" > $out/test.log 2>&1
rc=$?; tail -2 $out/test.log; [ $rc -eq 0 ] || exit $rc
run() {  # name size env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --size $n > $out/$name.json 2> $out/$name.err || return $?
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); p=d['policy']; print('$name', d['ms_per_step'], d['check'], d['residual_ratio'], p['main_cnt'])"
}
for rep in 1 2; do
  for n in 8192 16384 32768; do
    run n${n}_main_$rep $n GJ_NONE=0 || exit $?
    run n${n}_none_$rep $n GJ_MAIN_CNT=0 || exit $?
    run n${n}_all_$rep $n GJ_GLDS_CNT=3 || exit $?
  done
done
