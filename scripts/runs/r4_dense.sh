#!/bin/bash
# Dense (5 workgroups/CU) trailing update where CUs are reserved for the pivot chain: A/B at the
# reserved-CU configurations (N = 8192 / 16384 on one GPU; emulated p = 8 at N = 32768 and p = 4 / 8
# at N = 16384) and the unreserved N = 32768 one (unchanged by construction).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/dense
mkdir -p $o
for rep in 1 2; do
  for d in 0 1; do
    for n in 8192 16384; do
      GJ_DENSE_GEMM=$d timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 3 --no-residual > $o/b${n}_d${d}_$rep.json 2>&1 || exit $?
      python3 -c "import json; d=json.loads(open('$o/b${n}_d${d}_$rep.json').read().splitlines()[-1]); print('dense=$d n=$n rep=$rep', d['ms_per_step'], d['policy']['dense_gemm'])"
    done
  done
done
for d in 0 1; do
  GJ_DENSE_GEMM=$d timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct > $o/emu32k_d$d.txt 2>&1 || exit $?
  echo "dense=$d"; tail -2 $o/emu32k_d$d.txt
  GJ_DENSE_GEMM=$d timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --reps 2 --bw 50 --bcast direct > $o/emu16k_d$d.txt 2>&1 || exit $?
  tail -4 $o/emu16k_d$d.txt
done
