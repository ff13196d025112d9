#!/bin/bash
# Round-4 measurements (one box): one-GPU sizes after the live-candidate launches and the host-free
# p = 1 chain, then the p-rank emulation with the host-driven and the host-free (GJ_HOST_FREE=1,
# all-reduce panel pieces) chains at p > 1.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
o=gpurun_out/r4m
for n in 8192 16384; do
  timeout -k 10 200 python bench.py --size $n --steps 10 --warmup 3 > $o/b$n.json 2> $o/b$n.err || exit $?
  tail -1 $o/b$n.json | cut -c1-300
done
timeout -k 10 240 python bench.py --steps 5 --warmup 2 > $o/b32768.json 2> $o/b32768.err || exit $?
tail -1 $o/b32768.json | cut -c1-300
for hf in 0 1; do
  GJ_HOST_FREE=$hf timeout -k 10 300 python bench/bench_emulate.py --ranks 4 8 --size 16384 --reps 2 --bw 50 --bcast direct > $o/emu16k_hf$hf.txt 2>&1 || exit $?
  cat $o/emu16k_hf$hf.txt | tail -4
done
for hf in 0 1; do
  GJ_HOST_FREE=$hf timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct > $o/emu32k_hf$hf.txt 2>&1 || exit $?
  cat $o/emu32k_hf$hf.txt | tail -2
done
# the 32-CU reservation of the p = 8 ranks, re-checked now that no dead inverse workgroup is dispatched
for rc in 0 32; do
  GJ_RESERVE_CUS=$rc timeout -k 10 300 python bench/bench_emulate.py --ranks 8 --size 32768 --reps 1 --bw 50 --bcast direct > $o/emu32k_res$rc.txt 2>&1 || exit $?
  cat $o/emu32k_res$rc.txt | tail -2
done
