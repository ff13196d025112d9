#!/bin/bash
# CU footprint of the RCCL kernels of a p = 2 solve: kernel trace of the
# --same-gpu rehearsal (both rank processes on device 0), then the RCCL kernels' grid / LDS / VGPRs.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/rcclfp
mkdir -p $o
# N = 2048, one step: the socket transport is slow under the profiler; the log goes straight into
# gpurun_out/ so a long run is not taken for a hung one
timeout -k 10 170 rocprofv3 --kernel-trace -d $o -o run -- python3 bench.py --gpus 2 --same-gpu --size 2048 --steps 1 --warmup 0 --comm-timeout 60 > $o/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $o/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 scripts/rccl_footprint.py $(find $o -name "*.db") | tee $o/footprint.md
