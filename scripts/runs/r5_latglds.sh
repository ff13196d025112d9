#!/bin/bash
# GJ_LAT_GLDS A/B: the pivot chain's column updates on the LDS-DMA kernel vs the 64 x 32 latency tile.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/latglds
mkdir -p $o
for rep in 1 2; do
  for lat in 0 1; do
    GJ_LAT_GLDS=$lat timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=32768 lat=$lat', d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for lat in 0 1; do
    GJ_LAT_GLDS=$lat timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
    echo "emu16k lat=$lat"; grep -h '"p"' $o/emu.txt | cut -c1-120
  done
done
for lat in 0 1; do
  GJ_LAT_GLDS=$lat timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu32k lat=$lat"; grep -h '"p"' $o/emu.txt | cut -c1-120
done
