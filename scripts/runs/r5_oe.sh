#!/bin/bash
# owner_edits with 32-bit index math: engine tests, N = 8192 / 16384, N = 8192 trace.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/oe
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --size 8192 --steps 20 --warmup 5 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=8192', d['ms_per_step'])"
  timeout -k 10 200 python bench.py --size 16384 --steps 5 --warmup 2 --no-residual > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=16384', d['ms_per_step'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof8k -o run -- python3 bench.py --size 8192 --steps 5 --warmup 2 --no-residual > $o/prof8k.log 2>&1 || { tail -5 $o/prof8k.log; exit 1; }
python3 scripts/side_chain.py $o/prof8k/run_results.db | head -14
