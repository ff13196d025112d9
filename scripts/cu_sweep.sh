#!/bin/bash
cd $GRAFT_REPO_ROOT
for spec in "0 1" "8 1" "16 1" "32 1" "16 0"; do
  set -- $spec
  for s in 8192 16384; do
    GJ_RESERVE_CUS=$1 GJ_RESERVE_MODE=$2 timeout -k 10 120 python bench.py --size $s --steps 5 --warmup 1 --no-residual > /tmp/o.json 2>/dev/null || exit 1
    echo "$1 $2 $s $(python -c "import json;d=json.load(open('/tmp/o.json'));print(d['ms_per_step'])")" >> gpurun_out/cu.log
  done
  GJ_RESERVE_CUS=$1 GJ_RESERVE_MODE=$2 timeout -k 10 200 python bench/bench_emulate.py --ranks 8 4 --reps 2 2>/dev/null | sed "s/^/$1 $2 /" >> gpurun_out/cu.log || exit 1
done
GJ_RESERVE_CUS=16 GJ_RESERVE_MODE=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual 2>/dev/null | sed "s/^/16 1 /" >> gpurun_out/cu.log
