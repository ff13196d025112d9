#!/bin/bash
# Round 6: the chunk pass's LDS footprint on the reserved CUs (GJ_CHUNK_BUILD) at N = 8192 / 16384,
# driver-shaped runs (20/5), two alternating repetitions; profiles/chain_r6.md.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/chain
mkdir -p $out
for rep in 1 2; do
  for n in 8192 16384; do
    for b in 0 23 25; do
      GJ_CHUNK_BUILD=$b timeout -k 10 120 python3 bench.py --size $n > $out/b${n}_${b}_$rep.json 2> $out/b${n}_${b}_$rep.err || exit $?
      python3 -c "import json; d=json.loads(open('$out/b${n}_${b}_$rep.json').read().strip().splitlines()[-1]); print($n, $b, $rep, d['ms_per_step'], d['check'])"
    done
  done
done
