#!/bin/bash
# (Record of a measurement: the switch it toggles was removed with the rejected variant; rerunning it
# now measures the default three times.)
# Barrier-free per-wave staged LDS-DMA GEMM (GJ_GLDS_SOLO=3/4 stages) vs the default.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/solo
mkdir -p $o
for st in 3 4; do
  GJ_GLDS_SOLO=$st timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k gemm --timeout 120 --timeout-method thread > $o/tests$st.txt 2>&1
  rc=$?; tail -1 $o/tests$st.txt; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for w in 0 3 4; do
    for sh in "32768 8192 512" "4096 32768 1024" "8192 4096 256"; do
      GJ_GLDS_SOLO=$w timeout -k 10 120 python bench/gemm_probe.py $sh --variant glds --reps 20 --check > $o/g.json 2>&1 || exit $?
      echo "solo=$w $(tail -1 $o/g.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['M'], d['N'], d['K'], d['tflops'], d['rel_err'])")"
    done
  done
done
for rep in 1 2; do
  for w in 0 3; do
    for n in 32768 16384; do
      GJ_GLDS_SOLO=$w timeout -k 10 200 python bench.py --size $n --steps 3 --warmup 1 > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('solve solo=$w n=$n', d['ms_per_step'], d['check'])"
    done
  done
done
