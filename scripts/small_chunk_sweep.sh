#!/bin/bash
# Chunk width at pivot-chain-bound sizes (default CU reservation and depth).
cd "$(dirname "$0")/.." || exit 1
for cc in 0 2048 4096 8192; do
  timeout -k 10 100 python bench.py --size 8192 --chunk-cols $cc --steps 5 --warmup 2 --no-residual 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n8192 chunk $cc', d['ms_per_step'])" || exit 1
done
for cc in 0 4096 8192 16384; do
  timeout -k 10 100 python bench.py --size 16384 --chunk-cols $cc --steps 3 --warmup 1 --no-residual 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n16384 chunk $cc', d['ms_per_step'])" || exit 1
  timeout -k 10 200 python bench/bench_emulate.py --ranks 4 8 --size 16384 --chunk-cols $cc --reps 2 2>&1 | grep -v amdgpu.ids |
    python -c "import json,sys; [print('emu', json.loads(l)['p'], 'n16384 chunk $cc', json.loads(l)['seconds']) for l in sys.stdin if l.strip()]" || exit 1
done
