#!/bin/bash
# Round 6: tile A/B at the unreserved middle sizes, and emulated p = 4 under the final rule.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/mid128
mkdir -p $out
for rep in 1 2; do
  for n in 20480 24576; do
    for t in 64 0; do
      GJ_GLDS_TILE=$t timeout -k 10 200 python3 bench.py --size $n --steps 10 --warmup 3 > $out/b${n}_$t_$rep.json 2> $out/b${n}_${t}_$rep.err || exit $?
      python3 -c "import json; d=json.loads(open('$out/b${n}_$t_$rep.json').read().strip().splitlines()[-1]); print($n, 'tile', $t or 'auto', $rep, d['ms_per_step'], d['check'], d['policy']['gemm_tile'])"
    done
  done
done
timeout -k 10 300 python3 bench/bench_emulate.py --ranks 4 --size 32768 --bw 50 --bcast direct --reps 2 > $out/emu4.jsonl 2> $out/emu4.err || exit $?
cut -c1-200 $out/emu4.jsonl
