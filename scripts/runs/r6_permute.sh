#!/bin/bash
# Round 6: the 16-byte block permutation (the inverse's final row / column reordering): kernel
# test, then its time inside the N = 8192 and N = 32768 solves (kernel trace), then the driver's
# N = 8192 run.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/permute
mkdir -p $out
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "permute" > $out/test.log 2>&1
rc=$?; tail -2 $out/test.log; [ $rc -eq 0 ] || exit $rc
for n in 8192 32768; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof$n -o run -- python3 bench.py --size $n --steps 2 --warmup 0 > $out/prof$n.log 2>&1 || exit $?
  tail -1 $out/prof$n.log | cut -c1-160
  f=$(find $out/prof$n -name "*kernel_stats.csv" | head -1)
  grep -i "permute" $f || true
done
timeout -k 10 200 python3 bench.py --size 8192 > $out/b8192.json 2> $out/b8192.err || exit $?
cut -c1-200 $out/b8192.json
