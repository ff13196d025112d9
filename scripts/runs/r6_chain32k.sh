#!/bin/bash
# Round 6: the final-build trace at N = 32768 has the pivot chain critical again (the candidate
# inverse 3.5 ms per step in the solve, MAIN 95 % busy): the one-launch look-ahead skip removed a
# launch boundary where CUs drained.  2 x 2: skip on / off x register / co-resident inverse.
# Driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/chain32k
mkdir -p $out
for rep in 1 2; do
  for cfg in "s1c0 GJ_SKIP_COLS=1 GJ_BI_CORESIDENT=0" "s0c0 GJ_SKIP_COLS=0 GJ_BI_CORESIDENT=0" "s1c1 GJ_SKIP_COLS=1 GJ_BI_CORESIDENT=1" "s0c1 GJ_SKIP_COLS=0 GJ_BI_CORESIDENT=1"; do
    set -- $cfg
    name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py > $out/${name}_$rep.json 2> $out/${name}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/${name}_$rep.json').read().strip().splitlines()[-1]); print('$name', $rep, d['ms_per_step'], d['check'])"
  done
done
