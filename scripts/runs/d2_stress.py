"""Race screening of depth-2 panels at p > 1, N > 8192: jittered async virtual ranks on one GPU.

Each case runs once; a residual far above the depth-4 control marks an ordering problem."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402

for name, p, d, n, gen, jit in [("ctl d4", 8, 4, 8192, "absdiff", 30.0), ("d2 j30", 8, 2, 8192, "absdiff", 30.0),
                                ("d2 j100", 8, 2, 8192, "absdiff", 100.0), ("d2 rnd j30", 8, 2, 8448, "random", 30.0),
                                ("d2 p4 j30", 4, 2, 8448, "random", 30.0), ("d2 j0", 8, 2, 8192, "absdiff", 0.0),
                                ("d3 j30", 8, 3, 8192, "absdiff", 30.0), ("d2 j300", 8, 2, 8192, "absdiff", 300.0)]:
    g = gj.GaussJordan(block_size=60, ranks=p, device="gpu", comm="async", depth=d, jitter_us=jit)
    rep = g.run(n, gen=gen)
    print(name, p, d, n, gen, jit, rep["status"], rep["residual"], flush=True)
