#!/bin/bash
# Trailing-update GEMM occupancy A/B inside the solver (GJ_GLDS_STAGES: 2 = 4 WG/CU, 9 = 3 WG/CU).
#   STAGE_LIST="2 9" bash scripts/occupancy_ab.sh
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for st in ${STAGE_LIST:-2 9}; do
  echo "stages=$st"
  GJ_GLDS_STAGES=$st timeout -k 10 60 python bench/gemm_probe.py 32768 4096 512 --variant glds --check 2>&1 | grep -v amdgpu.ids || exit 1
  for s in 32768 8192; do
    out=gpurun_out/occ_${st}_${s}.json
    GJ_GLDS_STAGES=$st timeout -k 10 200 python bench.py --size $s --steps 2 --warmup 1 --no-residual > $out 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['n'], d['ms_per_step'])" $out || exit 1
  done
  GJ_GLDS_STAGES=$st timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
done
