#!/bin/bash
# Multi-process RCCL rehearsal on one GPU (bench.py --same-gpu: every rank its own process and RCCL
# communicators; RCCL picks its socket transport between ranks sharing a device), final build.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
o=gpurun_out/rccl
mkdir -p $o
timeout -k 10 300 python bench.py --size 8192 --steps 2 --warmup 1 > $o/p1.json 2>&1 || exit $?
tail -1 $o/p1.json | cut -c1-600
for p in 2 4; do
  timeout -k 10 600 python bench.py --gpus $p --same-gpu --size 8192 --steps 1 --warmup 1 > $o/p$p.json 2>&1 || exit $?
  tail -1 $o/p$p.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p=$p', d['ms_per_step'], d['residual_inf'], d['check'], d['comm'], d.get('rccl_transport'), d['policy'])"
done
