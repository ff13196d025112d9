#!/bin/bash
# Parametrised A/B runner (replaces round 1-2's one-off *_ab.sh / *_sweep.sh drivers).
#
#   bash scripts/ab.sh [-r REPS] [-t SECONDS] -v "label:ENV=V [ENV2=V2 ...]" [-v ...] -- command args...
#
# Runs `command args...` once per variant per repetition, variants interleaved (a, b, a, b, ...) so
# that box drift hits every variant alike.  Each run gets its variant's environment and its own
# `timeout -k 10 SECONDS`; every output line is prefixed with "label rep". A run that ends with a
# fault, an abort, a time limit or a signal (status > 1) stops the whole sweep.
#
# Examples (the A/B experiments cited in profiles/*.md are all of this form):
#   bash scripts/ab.sh -r 2 -v "ring:GJ_BCAST=ring" -v "direct:GJ_BCAST=direct" -- \
#        python bench/bench_emulate.py --ranks 8 --size 32768 --bw 50
#   bash scripts/ab.sh -v "res0:GJ_RESERVE_CUS=0" -v "res32:GJ_RESERVE_CUS=32" -- \
#        python bench.py --size 8192 --steps 5 --no-residual
#   bash scripts/ab.sh -v "d2:" -v "d4:" -- python bench.py --size 16384 --depth 2   (same env, args differ: use two calls)
cd "$(dirname "$0")/.." || exit 1
reps=1
secs=600
variants=()
while [ $# -gt 0 ]; do
  case "$1" in
    -r) reps=$2; shift 2 ;;
    -t) secs=$2; shift 2 ;;
    -v) variants+=("$2"); shift 2 ;;
    --) shift; break ;;
    *) echo "ab.sh: unknown option $1" >&2; exit 2 ;;
  esac
done
[ $# -gt 0 ] || { echo "ab.sh: no command" >&2; exit 2; }
[ ${#variants[@]} -gt 0 ] || variants=("default:")
for rep in $(seq 1 "$reps"); do
  for v in "${variants[@]}"; do
    label=${v%%:*}
    envs=${v#*:}
    # shellcheck disable=SC2086
    env $envs timeout -k 10 "$secs" "$@" 2>&1 | sed -u "s/^/$label $rep /"
    rc=${PIPESTATUS[0]}
    if [ "$rc" -gt 1 ]; then
      echo "ab.sh: $label rep $rep ended with status $rc; stopping" >&2
      exit "$rc"
    fi
  done
done
