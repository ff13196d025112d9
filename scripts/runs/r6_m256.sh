#!/bin/bash
# Round 6: block size 256 at the headline size with the 128 x 128 tile (driver command shape).
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/m256
mkdir -p $out
p() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], round(d['value']/1e3,2), d['check'], d['residual_ratio'], d['policy']['depth'], d['policy']['block_inverse'])"; }
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py > $out/m128_$rep.json 2> $out/m128_$rep.err || exit $?
  p $out/m128_$rep.json m128_$rep
  timeout -k 10 200 python3 bench.py --block 256 > $out/m256_$rep.json 2> $out/m256_$rep.err || exit $?
  p $out/m256_$rep.json m256_d4_$rep
  timeout -k 10 200 python3 bench.py --block 256 --depth 2 > $out/m256d2_$rep.json 2> $out/m256d2_$rep.err || exit $?
  p $out/m256d2_$rep.json m256_d2_$rep
done
