#!/bin/bash
# Parametrised GPU session runner (one gpurun call): every argument is one step
#     "name|seconds|command"
# run from the repo root under its own `timeout -k 10 seconds`, output in gpurun_out/<name>.log.
# A step that exits 1 (a test or check failure) does not stop the session; any other non-zero
# status (a fault, an abort, a time limit, a signal) ends it there: nothing more runs on the GPU.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc in $(( $(date +%s) - start )) s"
  tail -4 "gpurun_out/$name.log" | cut -c1-600
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit "$rc"
  fi
done
