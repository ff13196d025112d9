#!/bin/bash
# One GPU session: tests, then benches.  Stops at the first fault/abort/timeout (exit >= 124 or
# signal-like codes); a plain test failure (exit 1) does not stop the later steps.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
for spec in "$@"; do
  echo "== bench $spec"
  timeout -k 10 600 python bench.py $spec > gpurun_out/bench_$(echo $spec | tr ' -' '__').log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_$(echo $spec | tr ' -' '__').log
  ok $rc || exit $rc
done
