#!/bin/bash
# p = 8 rank (4096 rows, N = 32768) under the 100 GB/s model: the default (depth 8, 32 reserved CUs,
# register inverse) against no reservation + co-resident inverse at depth 4 / 8.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {
  timeout -k 10 300 env "$@" python bench/bench_emulate.py --ranks 8 --size 32768 --reps 2 --bw 100 $DEPTH > gpurun_out/p8co.log 2>&1 || { tail -5 gpurun_out/p8co.log; return 1; }
  grep -v amdgpu.ids gpurun_out/p8co.log | grep model_bw | sed "s/^/$* $DEPTH /" | cut -c1-170
}
for rep in 1 2; do
  DEPTH="" run GJ_NONE=1 || exit 1
  DEPTH="" run GJ_RESERVE_CUS=0 GJ_BI_CORESIDENT=1 || exit 1
  DEPTH="--depth 4" run GJ_RESERVE_CUS=0 GJ_BI_CORESIDENT=1 || exit 1
  DEPTH="--depth 6" run GJ_RESERVE_CUS=0 GJ_BI_CORESIDENT=1 || exit 1
done | tee gpurun_out/p8_co.log
