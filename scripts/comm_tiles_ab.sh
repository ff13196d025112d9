#!/bin/bash
# A/B: COMM-stream chunk-normalisation GEMMs on the narrow 128x64 tile (0) vs the small 64x32 tile (1).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for s in ${SIZES:-8192 16384 32768}; do
  for r in 1 2; do
    for v in 0 1; do
      GJ_COMM_SMALL_TILES=$v timeout -k 10 200 python bench.py --size $s --steps 5 --warmup 2 --no-residual > gpurun_out/ct_${v}_${s}_$r.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('small_tiles', sys.argv[2], d['config']['n'], d['ms_per_step'], 'ms')" gpurun_out/ct_${v}_${s}_$r.json $v || exit 1
    done
  done
done
if [ -n "$EMU" ]; then
  for v in 0 1; do
    GJ_COMM_SMALL_TILES=$v timeout -k 10 200 python bench/bench_emulate.py --ranks 4 8 --size 16384 2>/dev/null | sed "s/^/small_tiles $v /" || exit 1
  done
fi
