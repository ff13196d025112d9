#!/bin/bash
# Every BASELINE.json config that runs on one MI355X (one JSON summary line each).
cd "$(dirname "$0")/.." || exit 1
summ='import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][-1]); print(json.dumps({k: d[k] for k in ("ms_per_step","value","residual_inf","dtype")} | {"n": d["config"]["n"], "m": d["config"]["m"]}))'
run() { timeout -k 10 300 python bench.py "$@" 2>/dev/null | python -c "$summ" || exit 1; }
run --size 8192 --steps 5 --warmup 2
run --size 16384 --steps 3 --warmup 1
run --size 32768 --steps 3 --warmup 1
run --size 32768 --steps 3 --warmup 1 --dtype fp32
run --size 65536 --steps 1 --warmup 1 --dtype fp32
run --size 65536 --steps 1 --warmup 1 --dtype fp32 --block 256
timeout -k 10 300 python bench/bench_emulate.py --ranks 2 4 8 --reps 2 2>/dev/null || exit 1
timeout -k 10 300 python bench/bench_emulate.py --ranks 4 --size 16384 --reps 2 2>/dev/null || exit 1
