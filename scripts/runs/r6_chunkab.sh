#!/bin/bash
# Round 6: the chunk pass around the 128 x 128 default at N = 32768 (driver command each):
# its GEMM tile, the chunk width, and merged launches around the panel columns.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/chunkab
mkdir -p $out
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py $BARGS > $out/$name.json 2> $out/$name.err || exit $?
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['check'])"
}
for rep in 1 2; do
  BARGS="" run default_$rep GJ_NONE=0
  BARGS="" run ctile64_$rep GJ_CHUNK_TILE=64
  BARGS="--chunk-cols 16384" run chunk16k_$rep GJ_NONE=0
  BARGS="" run cskip_$rep GJ_CHUNK_SKIP=1
done
