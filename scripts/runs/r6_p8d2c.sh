#!/bin/bash
# Round 6: after refusing GJ_SPLIT=2 on the GPU at p > 1: the schedule-variant test 3 times
# standalone, then the whole GPU tier and smoke().
cd "$(dirname "$0")/../.."
out=gpurun_out/p8d2c
mkdir -p $out
for rep in 1 2 3; do
  timeout -k 10 180 python3 -u -m pytest -q --timeout 150 --timeout-method thread \
      "tests/test_gpu_engine.py::test_split_column_updates_bit_identical_on_gpu" > $out/r$rep.log 2>&1
  rc=$?
  echo "rep $rep rc $rc $(tail -1 $out/r$rep.log)"
  grep -E "^E +(AssertionError|RuntimeError|assert)" $out/r$rep.log | head -2 | cut -c1-400
  [ $rc -le 1 ] || exit $rc
done
bash scripts/runs/r6_tier.sh
