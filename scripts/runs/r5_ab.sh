#!/bin/bash
# Same-box A/B of this round's two schedule/kernel changes, interleaved over two repetitions:
#   GJ_SPLIT   : chain / deferred split of the look-ahead + in-panel column updates (engine)
#   GJ_GLDS_PEEL: peeled, stage-unrolled LDS-DMA trailing-update loop (2 stages; 3.3 = 3 stages)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/ab5
mkdir -p $o
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" > $o/b.json 2> $o/b.err || { echo "$label FAILED"; tail -5 $o/b.err; return 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('$label', d['ms_per_step'], d['policy'].get('split'))"
}
for rep in 1 2; do
  for n in 8192 16384; do
    for s in 0 1; do
      run "n=$n split=$s" GJ_SPLIT=$s timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 2 --no-residual || exit 1
    done
  done
done
for rep in 1 2; do
  for v in "0 0 2.3" "1 0 2.3" "1 1 2.3" "1 1 3.3"; do
    set -- $v
    run "n=32768 split=$1 peel=$2 build=$3" GJ_SPLIT=$1 GJ_GLDS_PEEL=$2 GJ_GLDS_BUILD=$3 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-residual || exit 1
  done
done
for b in 2.3 3.3; do
  for p in 0 1; do
    GJ_GLDS_BUILD=$b GJ_GLDS_PEEL=$p timeout -k 10 120 python bench/gemm_probe.py 32768 8192 512 --ldc 32768 --reps 30 > $o/g.json 2>&1 || exit $?
    echo "gemm alone build=$b peel=$p $(tail -1 $o/g.json)"
  done
done
for p in 0 1; do
  GJ_GLDS_PEEL=$p timeout -k 10 200 python bench.py --size 8192 --steps 10 --warmup 2 --no-residual > $o/b.json 2>&1 && python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=8192 peel=$p', d['ms_per_step'])"
done
# emulated p = 8 / 4 ranks at N = 16384 (the 2048 / 4096-row ranks), auto depth (2 on the
# 2048-row rank since round 5) against depth 4, split on / off: rank-0 time, comm-free and the
# direct-broadcast 50 GB/s model
for s in 1 0; do
  GJ_SPLIT=$s timeout -k 10 300 python bench/bench_emulate.py --ranks 8 4 --size 16384 --depth 0 4 --bw 50 --bcast direct --reps 2 > $o/emu_$s.txt 2>&1 || exit $?
  echo "== emulate split=$s"; tail -12 $o/emu_$s.txt
done
