#!/bin/bash
# Current-build p-rank emulation table (rank 0, N = 32768 and 16384): comm-free and the 50 / 100 /
# 200 GB/s communication-cost model, plus bench.py on one GPU for the p = 1 column.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 3 > gpurun_out/emu_final_p1.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('p1 32768', d['ms_per_step'], 'ms')" gpurun_out/emu_final_p1.json || exit 1
for n in 32768 16384; do
  timeout -k 10 500 python bench/bench_emulate.py --ranks 2 4 8 --size $n --reps 2 --bw 50 100 200 > gpurun_out/emu_final_$n.log 2>&1 || { tail -5 gpurun_out/emu_final_$n.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/emu_final_$n.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['p'], d['n'], d.get('model_bw_gbs', 'free'), d['seconds'], d.get('comm_hidden', ''))
"
done
