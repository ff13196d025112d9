#!/bin/bash
# Panel depth at pivot-chain-bound sizes (with the default CU reservation): 1 GPU and emulated p.
cd "$(dirname "$0")/.." || exit 1
for d in 2 4; do
  timeout -k 10 100 python bench.py --size 16384 --depth $d --steps 3 --warmup 1 --no-residual 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n16384 depth', d['config']['depth'], d['ms_per_step'])" || exit 1
done
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 16384 --depth 2 4 --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --size 8192 --depth 2 4 --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
