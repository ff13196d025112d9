#!/bin/bash
# Round 6: the final tier once returned a wrong inverse in
# test_split_column_updates_bit_identical_on_gpu[8-async-2] (p = 8 asynchronous virtual ranks,
# explicit depth 2: the configuration of the round-3 wrong inverse).  Bounded diagnostic: the same
# case 4 times with MAIN's non-temporal C (default) and 4 times without (GJ_MAIN_CNT=0),
# alternating; a wrong result is an assertion, not a GPU fault, so every run is recorded.
cd "$(dirname "$0")/../.."
out=gpurun_out/p8d2
mkdir -p $out
for rep in 1 2 3 4; do
  for c in 3 0; do
    GJ_MAIN_CNT=$c timeout -k 10 180 python3 -u -m pytest -q --timeout 150 --timeout-method thread \
        "tests/test_gpu_engine.py::test_split_column_updates_bit_identical_on_gpu[8-async-2]" > $out/c${c}_$rep.log 2>&1
    rc=$?
    echo "main_cnt $c rep $rep rc $rc $(tail -1 $out/c${c}_$rep.log)"
    # stop on anything but pass (0) / assertion failure (1)
    [ $rc -le 1 ] || exit $rc
  done
done
