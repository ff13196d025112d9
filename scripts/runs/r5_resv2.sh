#!/bin/bash
# N = 16384 without the CU reservation, now that the chain has the register-fed latency kernel and
# the merged launches (both gated on the reservation): is 32 CUs still the right default?
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/resv2
mkdir -p $o
run() {  # label depth env...
  local label=$1 depth=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --size 16384 --steps 5 --warmup 2 --depth $depth --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('$label depth=$depth', d['ms_per_step'])"
}
for rep in 1 2; do
  run default 0 GJ_X=0 || exit 1
  run r0 3 GJ_RESERVE_CUS=0 || exit 1
  run r0+lat 3 GJ_RESERVE_CUS=0 GJ_LAT_REG=1 || exit 1
  run r0+lat+skip 3 GJ_RESERVE_CUS=0 GJ_LAT_REG=1 GJ_SKIP_COLS=1 || exit 1
  run r0+lat+skip 4 GJ_RESERVE_CUS=0 GJ_LAT_REG=1 GJ_SKIP_COLS=1 || exit 1
done
