#!/bin/bash
# Round 6: chunk width around the 128 x 128 default at N = 32768 (driver command each), and the
# chunk pass's GEMM tile.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/chunkab2
mkdir -p $out
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py $BARGS > $out/$name.json 2> $out/$name.err || exit $?
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['check'], d['policy']['nchunks'], d['policy']['chunk_cols'])"
}
for rep in 1 2; do
  BARGS="" run default_$rep GJ_NONE=0
  BARGS="" run ctile64_$rep GJ_CHUNK_TILE=64
  BARGS="--chunk-cols 4096" run c4k_$rep GJ_NONE=0
  BARGS="--chunk-cols 6144" run c6k_$rep GJ_NONE=0
  BARGS="--chunk-cols 12288" run c12k_$rep GJ_NONE=0
done
