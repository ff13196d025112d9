#!/bin/bash
# Register-fed small fp64 GEMM for the chain's latency launches (GJ_LAT_KERNEL) A/B.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/latk
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "latency or row_blocks or skip or batch" > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {  # size steps warmup k
  GJ_LAT_REG=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 lat_reg=$4', d['ms_per_step'])"
}
for rep in 1 2; do for k in 0 1; do run 8192 20 5 $k || exit 1; done; done
for rep in 1 2; do for k in 0 1; do run 16384 5 2 $k || exit 1; done; done
for k in 0 1; do
  GJ_LAT_REG=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu16k lat_kernel=$k: $(grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
print(' '.join('%s/%s=%s' % (d['p'], d.get('bcast', 'free'), d['seconds']) for d in map(json.loads, sys.stdin)))")"
  GJ_LAT_REG=$k timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu32k lat_kernel=$k: $(grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
print(' '.join('%s/%s=%s' % (d['p'], d.get('bcast', 'free'), d['seconds']) for d in map(json.loads, sys.stdin)))")"
done
