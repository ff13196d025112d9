#!/bin/bash
# Round 6 closing: the driver's headline command (twice) with the clock sampler, two last in-solve
# A/Bs around the 128 x 128 tile (3 LDS stages, C loads before the first slices), the BASELINE sizes.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/final
mkdir -p $out
p() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], round(d['value']/1e3,2), d['check'], min(d['step_ms']), max(d['step_ms']))"; }
timeout -k 10 200 python3 scripts/smi_sample.py $out/smi_1.jsonl -- python3 bench.py > $out/b1.json 2> $out/b1.err || exit $?
p $out/b1.json default_1
timeout -k 10 200 env GJ_GLDS_BUILD=3.3 python3 bench.py > $out/s3.json 2> $out/s3.err || exit $?
p $out/s3.json stages3
timeout -k 10 200 env GJ_GLDS_COVL=0 python3 bench.py > $out/covl0.json 2> $out/covl0.err || exit $?
p $out/covl0.json covl0
timeout -k 10 200 python3 bench.py > $out/b2.json 2> $out/b2.err || exit $?
p $out/b2.json default_2
for n in 8192 16384; do
  timeout -k 10 120 python3 bench.py --size $n > $out/b$n.json 2> $out/b$n.err || exit $?
  p $out/b$n.json n$n
done
timeout -k 10 200 python3 bench.py --dtype fp32 > $out/f32.json 2> $out/f32.err || exit $?
p $out/f32.json fp32_32768
