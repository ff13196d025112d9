#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default twice.)
# 128 x 128 8-wave LDS-DMA tile (GJ_GLDS_WIDE=2/3 stages) vs the default 128 x 64 4-wave tile.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/wide
mkdir -p $o
GJ_GLDS_WIDE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k gemm --timeout 120 --timeout-method thread > $o/tests.txt 2>&1
rc=$?; tail -2 $o/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for w in 0 2 3; do
    for sh in "32768 8192 512" "4096 32768 1024" "8192 4096 256"; do
      GJ_GLDS_WIDE=$w timeout -k 10 120 python bench/gemm_probe.py $sh --variant glds --reps 20 --check > $o/g.json 2>&1 || exit $?
      echo "wide=$w $(tail -1 $o/g.json | cut -c1-160)"
    done
  done
done
for rep in 1 2; do
  for w in 0 2 3; do
    for n in 32768 16384; do
      GJ_GLDS_WIDE=$w timeout -k 10 200 python bench.py --size $n --steps 3 --warmup 1 > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('solve wide=$w n=$n', d['ms_per_step'], d['check'])"
    done
  done
done
