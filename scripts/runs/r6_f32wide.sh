#!/bin/bash
# Round 6: the fp32 128 x 256 LDS-DMA tile (numerics, alone, N = 32768 / 65536 A/B), then the
# emulated p = 2 / 4 / 8 ranks with the channel-footprint receive model.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/f32w
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    -k "tile256 or tile128 or glds" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for t in 64 0; do
    GJ_GLDS_TILE=$t timeout -k 10 120 python3 bench/gemm_probe.py 32768 8192 512 --ldc 32768 --dtype fp32 --variant glds --reps 20 >> $out/probe.jsonl 2>> $out/probe.err || exit $?
  done
done
cut -c1-200 $out/probe.jsonl
for rep in 1 2; do
  for t in 64 0; do
    GJ_GLDS_TILE=$t timeout -k 10 200 python3 bench.py --dtype fp32 > $out/b32k_${t}_$rep.json 2> $out/b32k_${t}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/b32k_${t}_$rep.json').read().strip().splitlines()[-1]); print('fp32 32768 tile', $t, $rep, d['ms_per_step'], d['check'])"
  done
done
for t in 64 0; do
  GJ_GLDS_TILE=$t timeout -k 10 300 python3 bench.py --dtype fp32 --size 65536 --gen randshift --rhs ones --steps 3 --warmup 1 > $out/cfg5_$t.json 2> $out/cfg5_$t.err || exit $?
  python3 -c "import json; d=json.loads(open('$out/cfg5_$t.json').read().strip().splitlines()[-1]); print('cfg5 tile', $t, d['ms_per_step'], d['check'], d['rhs']['final_relative_residual'])"
done
timeout -k 10 400 python3 bench/bench_emulate.py --ranks 2 4 8 --size 32768 --bw 50 100 --bcast direct --reps 2 \
    > $out/emu32k.jsonl 2> $out/emu32k.err || { tail -5 $out/emu32k.err; exit 1; }
cut -c1-200 $out/emu32k.jsonl
