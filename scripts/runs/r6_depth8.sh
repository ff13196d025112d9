#!/bin/bash
# Round 6: depth 8 (K = 1024: half the C traffic per flop, which the power-limited card would turn
# into clock) at N = 32768.  Depth 8 with 8192-column chunks gives the pivot chain 8 steps per 4 MAIN
# launches (the candidate inverse waits for a launch boundary, profiles/rocprof_n32768_r6_final.md);
# 4096-column chunks keep one launch per step.  Driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/depth8
mkdir -p $out
for rep in 1 2; do
  for cfg in "d4 --depth 4" "d8c4096 --depth 8 --chunk-cols 4096" "d8 --depth 8"; do
    set -- $cfg
    name=$1; shift
    timeout -k 10 300 python3 bench.py "$@" > $out/${name}_$rep.json 2> $out/${name}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/${name}_$rep.json').read().strip().splitlines()[-1]); print('$name', $rep, d['ms_per_step'], d['check'], d['residual_ratio'], d['policy']['nchunks'])"
  done
done
