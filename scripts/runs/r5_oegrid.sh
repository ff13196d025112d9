#!/bin/bash
# owner_edits grid cap (GJ_OE_GRID) at N = 8192 / 16384, plus the per-call kernel time from a trace.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/oegrid
mkdir -p $o
run() {  # size steps warmup grid
  GJ_OE_GRID=$4 timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup $3 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 grid=$4', d['ms_per_step'])"
}
for rep in 1 2; do for g in 256 64 16; do run 8192 20 5 $g || exit 1; done; done
for g in 256 64 16; do run 16384 5 2 $g || exit 1; done
for g in 256 16; do
  GJ_OE_GRID=$g timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof$g -o run -- python3 bench.py --size 8192 --steps 3 --warmup 1 --no-residual > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
  python3 - $o/prof$g/run_results.db $g <<'PY'
import sqlite3, sys
con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, end - start from kernels").fetchall()
d = sorted(t / 1e3 for n, t in rows if "owner_edits" in n)
print("grid", sys.argv[2], "owner_edits calls", len(d), "median us", d[len(d) // 2], "p10", d[len(d) // 10], "p90", d[9 * len(d) // 10])
PY
done
