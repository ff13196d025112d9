#!/bin/bash
# rocprofv3 kernel trace of bench.py at the pivot-chain-bound sizes + the SIDE-stream chain
# breakdown (scripts/side_chain.py) and the per-kernel summary (scripts/rocpd_summary.py).
#   bash scripts/prof_side.sh <tag> [sizes...]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=$1; shift
for n in ${@:-8192 16384}; do
  out=gpurun_out/prof_${tag}_$n
  mkdir -p "$out"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$out" -o run -- python3 bench.py --size $n --steps 1 --warmup 1 --no-residual > "$out/bench.log" 2>&1 || exit 1
  db=$(find "$out" -name "*.db" | head -1)
  python3 scripts/side_chain.py "$db" $(( n / 128 )) > "$out/side_chain.md" || exit 1
  python3 scripts/rocpd_summary.py "$db" > "$out/summary.md" 2>&1 || exit 1
  echo "== N=$n"; cat "$out/side_chain.md"; head -30 "$out/summary.md"
done
