#!/bin/bash
# Round 6: MAIN's chunk launch in two column halves (GJ_MAIN_SPLIT 1: the panel's first chunk, 2:
# every chunk): an extra launch boundary where a CU drains for the pivot chain's candidate inverse,
# which runs in lock-step with MAIN's launches at N = 32768 (profiles/rocprof_n32768_r6_final.md).
# Bit-identity on the GPU first (N = 5000), then the driver command, one box, alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/msplit
mkdir -p $out
timeout -k 10 200 python3 - > $out/ident.log 2>&1 <<'PY' || { cat $out/ident.log; exit 1; }
import os, numpy as np
import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix
A = generate_matrix(5000, "random", 3)
ref = gj.GaussJordan(block_size=128, device="gpu").inverse(A)
for sp in ("1", "2"):
    os.environ["GJ_MAIN_SPLIT"] = sp
    b = gj.GaussJordan(block_size=128, device="gpu").inverse(A)
    assert np.array_equal(ref, b), sp
print("bit-identical ok")
PY
cat $out/ident.log | tail -1
for rep in 1 2; do
  for sp in 0 1 2; do
    GJ_MAIN_SPLIT=$sp timeout -k 10 300 python3 bench.py > $out/s${sp}_$rep.json 2> $out/s${sp}_$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$out/s${sp}_$rep.json').read().strip().splitlines()[-1]); print('split $sp', $rep, d['ms_per_step'], d['check'], d['residual_ratio'])"
  done
done
