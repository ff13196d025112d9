#!/bin/bash
# Round 6, third closing run (the non-temporal C tile of the trailing update on top of the one-launch
# look-ahead skip with the 128 x 128 tile, the 16-byte permutation and the register candidate
# inverse on p > 1 ranks): the driver's headline
# command twice with the clock sampler, the BASELINE sizes, fp32, and the SCALE-shaped p = 2 / 3
# policies through real RCCL processes sharing the GPU with GJ_VERIFY=1.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/close3
mkdir -p $out
p() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], round(d['value']/1e3,2), d['check'], d.get('residual_inf'), min(d['step_ms']), max(d['step_ms']))"; }
timeout -k 10 200 python3 scripts/smi_sample.py $out/smi_1.jsonl -- python3 bench.py > $out/b1.json 2> $out/b1.err || exit $?
p $out/b1.json default_1
for n in 8192 16384; do
  timeout -k 10 120 python3 bench.py --size $n > $out/b$n.json 2> $out/b$n.err || exit $?
  p $out/b$n.json n$n
done
timeout -k 10 200 python3 bench.py --dtype fp32 > $out/f32.json 2> $out/f32.err || exit $?
p $out/f32.json fp32_32768
timeout -k 10 200 python3 scripts/smi_sample.py $out/smi_2.jsonl -- python3 bench.py > $out/b2.json 2> $out/b2.err || exit $?
p $out/b2.json default_2
GJ_VERIFY=1 timeout -k 10 400 python3 bench.py --gpus 2 --same-gpu --size 32768 --steps 1 --warmup 1 \
    > $out/same2_32768.json 2> $out/same2_32768.err || { tail -20 $out/same2_32768.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/same2_32768.json').read().strip().splitlines()[-1]); print('same2', d['ms_per_step'], d['check'], repr(d.get('residual_inf')), d['policy']['block_inverse'], d['policy']['gemm_tile'], d['policy']['skip_cols'])"
GJ_VERIFY=1 timeout -k 10 300 python3 bench.py --gpus 3 --same-gpu --size 8192 --steps 2 --warmup 1 \
    > $out/same3_8192.json 2> $out/same3_8192.err || { tail -20 $out/same3_8192.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/same3_8192.json').read().strip().splitlines()[-1]); print('same3', d['ms_per_step'], d['check'], d['bcast_tuning'])"
# the communication-cost model's rank 0 of p = 2 / 4 / 8 at N = 32768 and p = 8 at N = 16384
# (depth 4, the p > 1 default, and an explicit depth 2)
timeout -k 10 400 python3 bench/bench_emulate.py --ranks 2 4 8 --size 32768 --bw 50 100 --bcast direct --reps 2 \
    > $out/emu32k.jsonl 2> $out/emu32k.err || { tail -5 $out/emu32k.err; exit 1; }
cut -c1-220 $out/emu32k.jsonl
timeout -k 10 300 python3 bench/bench_emulate.py --ranks 8 --size 16384 --bw 50 --bcast direct --reps 2 \
    > $out/emu16k.jsonl 2> $out/emu16k.err || { tail -5 $out/emu16k.err; exit 1; }
cut -c1-220 $out/emu16k.jsonl
timeout -k 10 300 python3 bench/bench_emulate.py --ranks 8 --size 16384 --depth 2 --bw 50 --bcast direct --reps 2 \
    > $out/emu16k_d2.jsonl 2> $out/emu16k_d2.err || { tail -5 $out/emu16k_d2.err; exit 1; }
cut -c1-220 $out/emu16k_d2.jsonl
