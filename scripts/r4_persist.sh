#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default twice.)
# Resident-grid (persistent) LDS-DMA GEMM vs one workgroup per tile: alone and in the N = 32768 solve.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/persist
mkdir -p $o
for rep in 1 2; do
  for v in "0 2.3" "1024 2.3" "1280 2.5" "0 2.5"; do
    set -- $v
    GJ_GLDS_PERSIST=$1 GJ_GLDS_BUILD=$2 timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --variant glds --reps 20 --check > $o/g_$1_$2_$rep.json 2>&1 || exit $?
    echo "persist=$1 build=$2 $(tail -1 $o/g_$1_$2_$rep.json)"
  done
done
for rep in 1 2; do
  for pg in 0 1024; do
    GJ_GLDS_PERSIST=$pg timeout -k 10 200 python bench.py --steps 3 --warmup 1 > $o/b_$pg_$rep.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b_$pg_$rep.json').read().splitlines()[-1]); print('solve persist=$pg', d['ms_per_step'], d['check'])"
  done
done
