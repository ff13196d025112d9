#!/bin/bash
# Round 6: the co-resident 4-wave candidate inverse (72 KiB, GJ_BI_CORESIDENT=1) on one GPU beside
# the 2-stage 128 x 128 trailing-update tile (34 KiB x 3 per CU: one retiring tile makes room),
# at the sizes without a CU reservation, and at N = 16384 without the reservation.  Round 4
# measured it slower on one GPU with the 3-stage tiles, where two had to retire.
# Driver-shaped runs, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/coresident
mkdir -p $out
run() {  # name size env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --size $n > $out/$name.json 2> $out/$name.err || return $?
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); p=d['policy']; print('$name', d['ms_per_step'], d['check'], d['residual_ratio'], p['reserve_cus'], p['block_inverse'], p['gemm_tile'])"
}
for rep in 1 2; do
  run n16384_def_$rep 16384 GJ_NONE=0 || exit $?
  run n16384_co0_$rep 16384 GJ_RESERVE_CUS=0 GJ_BI_CORESIDENT=1 || exit $?
  run n20480_def_$rep 20480 GJ_NONE=0 || exit $?
  run n20480_co_$rep 20480 GJ_BI_CORESIDENT=1 || exit $?
  run n24576_def_$rep 24576 GJ_NONE=0 || exit $?
  run n24576_co_$rep 24576 GJ_BI_CORESIDENT=1 || exit $?
  run n32768_def_$rep 32768 GJ_NONE=0 || exit $?
  run n32768_co_$rep 32768 GJ_BI_CORESIDENT=1 || exit $?
done
