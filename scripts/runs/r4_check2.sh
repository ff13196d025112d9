#!/bin/bash
# GPU test tier (whole, not stopping at the first failure), the default headline bench and the
# N = 16384 / 8192 benches.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/c2/gputests.txt 2>&1
rc=$?; echo "tests_rc=$rc" >> gpurun_out/c2/gputests.txt; tail -3 gpurun_out/c2/gputests.txt
[ $rc -le 1 ] || exit $rc
for n in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --size $n --steps 5 --warmup 2 > gpurun_out/c2/bench_$n.txt 2>&1
  r=$?; tail -1 gpurun_out/c2/bench_$n.txt | cut -c1-400; [ $r -eq 0 ] || exit $r
done
