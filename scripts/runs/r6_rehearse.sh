#!/bin/bash
# Round 6: SCALE-shaped p = 2 policy through real RCCL processes on one GPU (verify on), BASELINE
# config 5 as a refined fp32 solve, and the policy-cliff sweep.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/reh
mkdir -p $out
GJ_VERIFY=1 timeout -k 10 400 python3 bench.py --gpus 2 --same-gpu --size 32768 --steps 1 --warmup 1 \
    > $out/same2_32768.json 2> $out/same2_32768.err || { tail -20 $out/same2_32768.err; exit 1; }
cut -c1-300 $out/same2_32768.json
GJ_VERIFY=1 timeout -k 10 300 python3 bench.py --gpus 3 --same-gpu --size 8192 --steps 2 --warmup 1 \
    > $out/same3_8192.json 2> $out/same3_8192.err || { tail -20 $out/same3_8192.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/same3_8192.json').read().strip().splitlines()[-1]); print(d['bcast_tuning'])"
timeout -k 10 300 python3 bench.py --dtype fp32 --size 65536 --gen randshift --rhs ones --steps 2 --warmup 1 \
    > $out/cfg5.json 2> $out/cfg5.err || { tail -20 $out/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/cfg5.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['rhs'])"
timeout -k 10 900 python3 scripts/policy_sweep.py $out/sweep.jsonl > $out/sweep.md 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 1; }
tail -24 $out/sweep.md
