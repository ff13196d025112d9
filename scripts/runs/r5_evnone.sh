#!/bin/bash
# GJ_EVENT_RELEASE=none over the whole GPU tier, then N = 32768 system vs none.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/evnone
mkdir -p $o
GJ_EVENT_RELEASE=none timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputests.txt 2>&1
rc=$?
tail -3 $o/gputests.txt
[ $rc -eq 0 ] || exit $rc
run() {  # size steps warmup mode [extra]
  GJ_EVENT_RELEASE=$4 timeout -k 10 300 python bench.py --size $1 --steps $2 --warmup $3 $5 > $o/b.json 2>&1 || { tail -5 $o/b.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/b.json').read().splitlines()[-1]); print('n=$1 ev=$4', d['ms_per_step'], d.get('check', ''), d.get('residual_inf', ''))"
}
GJ_EVENT_RELEASE=none timeout -k 10 300 python bench.py > $o/def.json 2>&1 || { tail -5 $o/def.json; exit 1; }
tail -1 $o/def.json
for rep in 1 2; do for k in system none; do run 32768 3 1 $k --no-residual || exit 1; done; done
