#!/bin/bash
# Whole GPU tier on the round-5 defaults, the three one-GPU sizes, fp32 N = 32768, and a kernel trace
# of N = 8192 (the pivot chain per step) for profiles/.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/c5
mkdir -p $o
timeout -k 10 780 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/gputests.txt 2>&1
rc=$?; echo "tests_rc=$rc" >> $o/gputests.txt; tail -4 $o/gputests.txt
[ $rc -le 1 ] || exit $rc
for v in "32768 5" "16384 10" "8192 20"; do
  set -- $v
  timeout -k 10 200 python bench.py --size $1 --steps $2 --warmup 2 > $o/b$1.json 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$o/b$1.json').read().splitlines()[-1]); print('n=$1', d['ms_per_step'], d['value'], d['check'], d['residual_ratio'])"
done
timeout -k 10 200 python bench.py --dtype fp32 --steps 3 --warmup 1 > $o/bf32.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('$o/bf32.json').read().splitlines()[-1]); print('fp32 n=32768', d['ms_per_step'], d['value'], d['check'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof8k -o run -- python3 bench.py --size 8192 --steps 5 --warmup 2 --no-residual > $o/prof8k.log 2>&1
echo "rocprof rc=$?"
