#!/bin/bash
# BASELINE config 3 region: emulated p = 4 / 8 at N = 16384, depth 4 / 6 / 8, 50 GB/s direct model.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/cfg3
mkdir -p $o
timeout -k 10 600 python bench/bench_emulate.py --ranks 4 8 --size 16384 --depth 4 6 8 --reps 2 --bw 50 --bcast direct > $o/emu.txt 2>&1 || exit $?
grep '"seconds"' $o/emu.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('emu', d['p'], d['n'], d['depth'], d.get('bcast', 'free'), d['seconds'])"
