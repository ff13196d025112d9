#!/bin/bash
# Split v2 A/B: the used rows' column updates deferred to MAIN (GJ_SPLIT=2), the chain's row-selected
# updates on the LDS-DMA kernel, and the chain's column updates on the LDS-DMA kernel (GJ_LAT_GLDS=1).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/split2
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k row_blocks \
  tests/test_gpu_engine.py -k "row_blocks or split" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
run() {  # size steps warmup split lat
  GJ_SPLIT=$4 GJ_LAT_GLDS=$5 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 split=$4 lat=$5', d['ms_per_step'])"
}
for rep in 1 2; do
  for cfg in "0 0" "0 1" "2 0" "2 1" "1 1"; do run 8192 20 5 $cfg || exit 1; done
done
for rep in 1 2; do
  for cfg in "0 0" "0 1" "2 0" "2 1"; do run 16384 5 2 $cfg || exit 1; done
done
for cfg in "0 0" "2 1"; do
  GJ_SPLIT=${cfg% *} GJ_LAT_GLDS=${cfg#* } timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "emu split/lat=$cfg"; grep -h '"p"' $o/emu.txt | cut -c1-200
done
