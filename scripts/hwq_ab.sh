#!/bin/bash
# A/B of the hardware-queue count (GPU_MAX_HW_QUEUES 4 = the box default, 8, 16 = runtime_env.py).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for q in 4 8 16; do
  for n in 8192 16384 32768; do
    GJ_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --size $n --steps 3 --no-residual > gpurun_out/hwq.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" gpurun_out/hwq.json "rep=$rep queues=$q n=$n" || exit 1
  done
done
done
