"""fp32 engine with large candidate blocks: relative error vs numpy per block-inverse kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402
from mpi_jordan_crazy_acceleration_amd import load_native  # noqa: E402
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix  # noqa: E402

C = load_native()
n = 1500
A = generate_matrix(n, "random", 17)
ref = np.linalg.inv(A)
for m, var in [(128, "panel"), (200, "panel"), (300, "panel"), (300, "generic"), (520, "panel"), (520, "generic")]:
    for dt in ("fp32", "fp64"):
        C.set_block_inverse_variant(var)
        try:
            rep = gj.GaussJordan(block_size=m, ranks=1, device="gpu", dtype=dt).run(n, input=A, keep_inverse=True)
            inv = rep["inverse"]
            print(m, var, dt, "status", rep["status"], "rel", float(np.abs(inv - ref).max() / np.abs(ref).max()),
                  "resid", rep["residual"], flush=True)
        finally:
            C.set_block_inverse_variant("panel")
