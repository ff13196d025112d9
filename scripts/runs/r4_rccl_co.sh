#!/bin/bash
# The co-resident candidate inverse with its fused selection (the default on ranks without a CU
# reservation, i.e. p = 2 / 4 at N = 32768) through the multi-process RCCL path: p = 1 vs p = 2
# (--same-gpu), forced at N = 8192.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/rcclco
mkdir -p $o
GJ_BI_CORESIDENT=1 timeout -k 10 300 python bench.py --size 8192 --steps 1 --warmup 1 > $o/p1.json 2>&1 || exit $?
tail -1 $o/p1.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p=1', d['ms_per_step'], repr(d['residual_inf']), d['check'], d['policy']['block_inverse'])"
GJ_BI_CORESIDENT=1 timeout -k 10 600 python bench.py --gpus 2 --same-gpu --size 8192 --steps 1 --warmup 1 > $o/p2.json 2>&1 || exit $?
tail -1 $o/p2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p=2', d['ms_per_step'], repr(d['residual_inf']), d['check'], d['policy']['block_inverse'], d.get('rccl_transport'))"
