#!/bin/bash
# fp32 peeled LDS-DMA trailing update (GJ_GLDS32_BUILD 2.4 default / 2.3 / 3.3, GJ_GLDS_PEEL=0 the
# round-4 loop) alone and in the N = 32768 / 65536 fp32 solves; the dense (5-per-CU) build under the
# p = 8 reservation with the peeled loop; N = 8192 3.3 vs dense.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/fp32r5
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -k "deep_auto or elimination_extras or fp32" --timeout 120 --timeout-method thread > $o/tests.txt 2>&1
rc=$?; tail -2 $o/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in "1 2.4" "1 2.3" "1 3.3" "0 2.4"; do
  set -- $v
  GJ_GLDS_PEEL=$1 GJ_GLDS32_BUILD=$2 timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --dtype fp32 --ldc 32768 --reps 30 > $o/g.json 2>&1 || exit $?
  echo "fp32 gemm peel=$1 build=$2 $(tail -1 $o/g.json | cut -c1-200)"
done
for rep in 1 2; do
  for v in "1 2.4" "1 3.3" "0 2.4"; do
    set -- $v
    GJ_GLDS_PEEL=$1 GJ_GLDS32_BUILD=$2 timeout -k 10 200 python bench.py --dtype fp32 --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('fp32 n=32768 peel=$1 build=$2', d['ms_per_step'])"
  done
done
timeout -k 10 300 python bench.py --dtype fp32 --size 65536 --steps 1 --warmup 1 > $o/b65.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('$o/b65.json').read().splitlines()[-1]); print('fp32 n=65536', d['ms_per_step'], d['check'], d['residual_ratio'])"
for rep in 1 2; do
  for dn in 0 1; do
    GJ_DENSE_GEMM=$dn timeout -k 10 200 python bench.py --size 8192 --steps 20 --warmup 2 --no-residual > $o/b.json 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=8192 dense=$dn', d['ms_per_step'])"
  done
done
for dn in 1 0; do
  GJ_DENSE_GEMM=$dn timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu_$dn.txt 2>&1 || exit $?
  echo "== p=8 N=32768 dense=$dn"; grep -h '"p"' $o/emu_$dn.txt | cut -c1-200
done
# every non-latency GEMM on the LDS-DMA kernel (the COMM normalisations and the look-ahead update
# too), against the shape rule
for rep in 1 2; do
  for n in 8192 16384; do
    for v in auto glds; do
      GJ_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 --no-residual > $o/b.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$n variant=$v', d['ms_per_step'])"
    done
  done
done
for v in auto glds; do
  GJ_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual > $o/b.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=32768 variant=$v', d['ms_per_step'])"
done
