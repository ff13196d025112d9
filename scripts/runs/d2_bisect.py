"""Replay of the GPU-tier sequence that once failed at p = 8, n = 8192, m = 60 with depth 2 (temporary):
the golden-residual file's runs in order, the last one at depth 2, three times."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402

for rep_i in range(3):
    for m in (30, 60, 90, 120, 240):
        r = gj.GaussJordan(block_size=m, ranks=8, device="gpu", comm="async", jitter_us=20.0).run(2048, gen="absdiff")
        print(rep_i, "n2048", m, r["status"], r["residual"], flush=True)
    for n in (4096, 8192):
        for p in (2, 4, 8):
            d = 2 if (n == 8192 and p == 8) else 0
            r = gj.GaussJordan(block_size=60, ranks=p, device="gpu", comm="async", depth=d).run(n, gen="absdiff")
            print(rep_i, "m60", n, p, d, r["status"], r["residual"], flush=True)
