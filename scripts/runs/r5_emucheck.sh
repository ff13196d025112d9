#!/bin/bash
# Emulated p = 4 / 8 ranks: the round's late defaults on / off, one box, interleaved.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/emucheck
mkdir -p $o
emu() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 0 --bw 50 --bcast direct --reps 1 > $o/emu.txt 2>&1 || { tail -5 $o/emu.txt; exit 1; }
  echo "$label: $(grep -h '"p"' $o/emu.txt | python3 -c "
import sys, json
print(' '.join('%s/%s=%s' % (d['p'], d.get('bcast', 'free'), d['seconds']) for d in map(json.loads, sys.stdin)))")"
}
for rep in 1 2; do
  emu "default" GJ_X=0 || exit 1
  emu "covl0" GJ_GLDS_COVL=0 || exit 1
  emu "skip0" GJ_SKIP_COLS=0 || exit 1
done
