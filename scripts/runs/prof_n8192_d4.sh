#!/bin/bash
# rocprofv3 kernel traces of N = 8192 at depth 4 (32 / 64 reserved CUs) and the default depth 2,
# for scripts/side_chain.py (profiles/side_chain_r3.md).  One bench step after one warm-up.
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
set -o pipefail
run() {  # name, env..., -- bench args
  local name=$1; shift
  local out=gpurun_out/prof_$name
  mkdir -p "$out"
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d "$out" -o run -- python3 bench.py --size 8192 --steps 1 --warmup 1 --no-residual $BARGS > "$out/bench.log" 2>&1
}
BARGS="--depth 4" run n8192_d4_r32 GJ_RESERVE_CUS=32 && \
BARGS="--depth 4" run n8192_d4_r64 GJ_RESERVE_CUS=64 && \
BARGS="--depth 2" run n8192_d2_r32 GJ_RESERVE_CUS=32 && \
for n in n8192_d4_r32 n8192_d4_r64 n8192_d2_r32; do echo "== $n"; grep '^{' gpurun_out/prof_$n/bench.log | cut -c1-200; d=${n#n8192_d}; d=${d%%_*}; python3 scripts/side_chain.py gpurun_out/prof_$n/run_results.db 64 $d; done
