#!/bin/bash
# CU reservation for the pivot chain (GJ_RESERVE_CUS, mode 0 = the first n CUs) across regimes.
cd "$(dirname "$0")/.." || exit 1
emu() {  # ranks size reserve
  GJ_RESERVE_CUS=$3 GJ_RESERVE_MODE=0 timeout -k 10 300 python bench/bench_emulate.py --ranks $1 --size $2 --reps 2 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('emu p=$1 n=$2 reserve=$3', d['seconds'])" || exit 1
}
one() {  # size reserve
  GJ_RESERVE_CUS=$2 GJ_RESERVE_MODE=0 timeout -k 10 200 python bench.py --size $1 --steps 3 --warmup 1 --no-residual 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('p=1 n=$1 reserve=$2', d['ms_per_step'])" || exit 1
}
for r in ${RES_LIST:-0 32 48 64}; do
  one 8192 $r || exit 1
  emu 4 16384 $r || exit 1
  emu 8 16384 $r || exit 1
  emu 2 16384 $r || exit 1
  emu 8 32768 $r || exit 1
done
