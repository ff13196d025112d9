#!/bin/bash
# Does a candidate inverse that starts inside a running trailing update (co-resident 4-wave form)
# make deeper panels (K = 1024 trailing updates) pay at p = 1?  N = 32768 and 16384.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/codepth
mkdir -p $o
run() {  # tag n depth co
  GJ_BI_CORESIDENT=$4 timeout -k 10 200 python bench.py --size $2 --depth $3 --steps 3 --warmup 1 --no-residual > $o/$1.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/$1.json').read().splitlines()[-1]); print('$1', d['ms_per_step'], d['policy']['depth'])"
}
for rep in 1 2; do
  run d4_co0_32k_$rep 32768 4 0
  run d4_co1_32k_$rep 32768 4 1
  run d8_co0_32k_$rep 32768 8 0
  run d8_co1_32k_$rep 32768 8 1
  run d6_co1_32k_$rep 32768 6 1
done
run d4_co0_16k 16384 4 0
run d4_co1_16k 16384 4 1
run d8_co1_16k 16384 8 1
