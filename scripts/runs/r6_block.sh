#!/bin/bash
# Round 6: block size m at the chain-bound sizes (driver-shaped 20/5 runs; m is the reference's CLI
# argument, the pivot-block granularity).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/block
mkdir -p $out
for rep in 1 2; do
  for n in 8192 16384; do
    for m in 128 192 256; do
      timeout -k 10 200 python3 bench.py --size $n --block $m > $out/b${n}_${m}_$rep.json 2> $out/b${n}_${m}_$rep.err || exit $?
      python3 -c "import json; d=json.loads(open('$out/b${n}_${m}_$rep.json').read().strip().splitlines()[-1]); print($n, $m, $rep, d['ms_per_step'], d['check'], d['residual_ratio'], d['policy']['depth'], d['policy']['reserve_cus'], d['policy']['block_inverse'])"
    done
  done
done
