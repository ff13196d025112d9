#!/bin/bash
# LDS-DMA GEMM main loop with its order pinned (sched_barrier: next slice's DMA issued first, all 16
# MFMAs of the slice before the vmcnt wait + barrier) vs the compiler's order (GJ_GLDS_PIN=0, which
# sank half of the MFMAs below the wait: the DMA had 8 MFMAs of cover instead of 16).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/pin
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k gemm --timeout 120 --timeout-method thread > $o/tests.txt 2>&1
rc=$?; tail -1 $o/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for pin in 0 1; do
    for b in 2.3 2.5; do
      for sh in "32768 8192 512" "4096 32768 1024" "8192 4096 256"; do
        GJ_GLDS_PIN=$pin GJ_GLDS_BUILD=$b timeout -k 10 120 python bench/gemm_probe.py $sh --variant glds --reps 20 --check > $o/g.json 2>&1 || exit $?
        echo "pin=$pin build=$b $(tail -1 $o/g.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['M'], d['N'], d['K'], d['tflops'], d['rel_err'])")"
      done
    done
  done
done
for rep in 1 2; do
  for pin in 0 1; do
    for n in 32768 16384 8192; do
      st=5; [ $n = 32768 ] && st=3
      GJ_GLDS_PIN=$pin timeout -k 10 200 python bench.py --size $n --steps $st --warmup 1 > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('solve pin=$pin n=$n', d['ms_per_step'], d['check'])"
    done
  done
done
