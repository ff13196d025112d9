#!/bin/bash
# Round 6: the 128 x 128 LDS-DMA trailing-update tile -- numerics, alone, in the solve (A/B on one
# box, driver command) with clock/power sampling; and the no-fence reproducer under GJ_VERIFY.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/t128
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    -k "tile128 or peeled" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  for cfg in "64 33" "128 33" "128 23" "128 32"; do
    set -- $cfg
    GJ_GLDS_TILE=$1 GJ_GLDS_BUILD=${2:0:1}.${2:1:1} timeout -k 10 120 python3 bench/gemm_probe.py 32768 8192 512 \
        --ldc 32768 --reps 20 >> $out/probe.jsonl 2>> $out/probe.err || exit $?
  done
done
cat $out/probe.jsonl
GJ_EVENT_RELEASE=none GJ_VERIFY=1 timeout -k 10 300 python3 scripts/runs/r6_nofence.py > $out/nofence.jsonl 2> $out/nofence.err || exit $?
cut -c1-600 $out/nofence.jsonl
for rep in 1 2; do
  for t in 64 128; do
    GJ_GLDS_TILE=$t timeout -k 10 300 python3 scripts/smi_sample.py $out/smi_${t}_$rep.jsonl -- \
        python3 bench.py > $out/b${t}_$rep.json 2> $out/b${t}_$rep.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$out/b${t}_$rep.json').read().strip().splitlines()[-1]); print($t, d['ms_per_step'], d['check'], min(d['step_ms']), max(d['step_ms']))"
  done
done
