#!/bin/bash
# Same-box A/B of the round-3 build (ab/r3, a worktree of 983d846 built in place) against this tree:
# bench.py at N = 8192 / 16384 / 32768, interleaved r3, r4, r3, r4.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/ab
mkdir -p $o
for n in 8192 16384 32768; do
  steps=10; [ $n -eq 32768 ] && steps=4
  for rep in 1 2; do
    for who in r3 r4; do
      dir=.; [ $who = r3 ] && dir=ab/r3
      timeout -k 10 240 python $dir/bench.py --size $n --steps $steps --warmup 2 --no-residual > $o/${who}_${n}_$rep.json 2> $o/${who}_${n}_$rep.err || exit $?
      python3 -c "import json,sys; d=json.loads(open('$o/${who}_${n}_$rep.json').read().splitlines()[-1]); print('$who', $n, $rep, d['ms_per_step'], d['value'])"
    done
  done
done
# in-solve residency trade of the trailing-update GEMM, re-measured after the chain got lighter
for b in 2.3 2.5 3.3; do
  GJ_GLDS_BUILD=$b timeout -k 10 240 python bench.py --steps 4 --warmup 2 --no-residual > $o/glds_$b.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/glds_$b.json').read().splitlines()[-1]); print('glds $b', d['ms_per_step'])"
  GJ_GLDS_BUILD=$b timeout -k 10 120 python bench.py --size 16384 --steps 8 --warmup 2 --no-residual > $o/glds16k_$b.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/glds16k_$b.json').read().splitlines()[-1]); print('glds16k $b', d['ms_per_step'])"
done
bash scripts/gemm_stall_pmc.sh
