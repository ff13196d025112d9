#!/bin/bash
# Round 6: broadcast / trailing-update chunk width at the chain-bound sizes (driver-shaped 20/5
# runs, two alternating repetitions).  The look-ahead rows of panel v wait for MAIN's update of
# panel v-1 over the chunk that holds panel v+1's columns; narrower chunks shorten that wait.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/chunk8k
mkdir -p $out
for rep in 1 2; do
  for cfg in "8192 0" "8192 2048" "8192 1024" "8192 2816" "16384 0" "16384 4096" "16384 2048"; do
    set -- $cfg
    n=$1; c=$2
    timeout -k 10 200 python3 bench.py --size $n --chunk-cols $c > $out/c${n}_${c}_$rep.json 2> $out/c${n}_${c}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/c${n}_${c}_$rep.json').read().strip().splitlines()[-1]); print($n, $c, $rep, d['ms_per_step'], d['check'], d['residual_ratio'], d['policy']['chunk_cols'])"
  done
done
