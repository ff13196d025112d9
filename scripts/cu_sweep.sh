#!/bin/bash
# CU reservation for the pivot path x trailing-update GEMM occupancy (GJ_GLDS_STAGES: 6 = 2 stages at
# 5 WG/CU, 2 = 2 stages at 4 WG/CU).  One line per run in gpurun_out/cu.log.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for st in ${STAGE_LIST:-6 2}; do
  for spec in ${RESERVE_LIST:-"0:0" "8:0" "16:0" "24:0"}; do
    n=${spec%%:*}; mode=${spec##*:}
    export GJ_GLDS_STAGES=$st GJ_RESERVE_CUS=$n GJ_RESERVE_MODE=$mode
    r1=$(timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-residual 2>/dev/null | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    r8=$(timeout -k 10 200 python bench/bench_emulate.py --ranks 8 4 --reps 1 2>/dev/null | python -c "import json,sys;print(' '.join(str(json.loads(l)['seconds']) for l in sys.stdin))") || exit 1
    echo "stages=$st reserve=$n mode=$mode n32768_ms=$r1 emu8,emu4_s=$r8" | tee -a gpurun_out/cu.log
  done
done
