#!/bin/bash
# Round 6, closing-build measurements of the tile-128 default at N = 32768: the XCD group and panel
# depth around it (driver command each), then a rocprofv3 kernel trace of a short run.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/p128
mkdir -p $out
for g in 4 2 8; do
  GJ_GLDS_GROUP=$g timeout -k 10 200 python3 bench.py > $out/g$g.json 2> $out/g$g.err || exit $?
  python3 -c "import json; d=json.loads(open('$out/g$g.json').read().strip().splitlines()[-1]); print('group $g', d['ms_per_step'], d['check'])"
done
timeout -k 10 200 python3 bench.py --depth 8 > $out/d8.json 2> $out/d8.err || exit $?
python3 -c "import json; d=json.loads(open('$out/d8.json').read().strip().splitlines()[-1]); print('depth 8', d['ms_per_step'], d['check'])"
timeout -k 10 200 python3 bench.py > $out/g4b.json 2> $out/g4b.err || exit $?
python3 -c "import json; d=json.loads(open('$out/g4b.json').read().strip().splitlines()[-1]); print('group 4 again', d['ms_per_step'], d['check'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $out/prof.log 2>&1 || exit $?
tail -1 $out/prof.log | cut -c1-200
