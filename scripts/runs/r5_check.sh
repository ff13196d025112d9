#!/bin/bash
# Round 5 check: whole GPU tier (GJ_VERIFY on in the multi-rank tests), the residual gate at the
# three one-GPU sizes (clean must pass, a corrupted late step at N = 8192 must fail), and the
# --same-gpu p = 2 rehearsal (two communicators, then one) with its profiled-solve record.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/r5c
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/gputests.txt 2>&1
rc=$?; echo "tests_rc=$rc" >> $o/gputests.txt; tail -5 $o/gputests.txt
[ $rc -le 1 ] || exit $rc
for n in 8192 16384 32768; do
  timeout -k 10 300 python bench.py --size $n --steps 3 --warmup 1 > $o/gate_$n.json 2> $o/gate_$n.err
  r=$?; python3 -c "import json; d=json.loads(open('$o/gate_$n.json').read().splitlines()[-1]); print('n=$n', d['ms_per_step'], d['check'], d['residual_inf'], d['residual_ratio'], d['norm_inv_inf'])"
  [ $r -eq 0 ] || exit $r
done
GJ_TEST_CORRUPT=0:60 timeout -k 10 300 python bench.py --size 8192 --steps 1 --warmup 0 > $o/corrupt.json 2> $o/corrupt.err
echo "corrupt rc=$? (2 expected)"; tail -c 600 $o/corrupt.err
timeout -k 10 300 python bench.py --gpus 2 --same-gpu --size 4096 --steps 2 --warmup 1 --comm-timeout 60 > $o/same2.json 2> $o/same2.err || exit $?
GJ_ONE_COMM=1 timeout -k 10 300 python bench.py --gpus 2 --same-gpu --size 4096 --steps 2 --warmup 1 --comm-timeout 60 > $o/same2_one.json 2> $o/same2_one.err || exit $?
python3 - <<'PY'
import json
for f in ("gpurun_out/r5c/same2.json", "gpurun_out/r5c/same2_one.json"):
    d = json.loads(open(f).read().splitlines()[-1])
    print(f, d["ms_per_step"], d["comm"], d["comm_mode"], d["residual_inf"], d.get("phases_ms_max"), d.get("profiled_solve"))
PY
