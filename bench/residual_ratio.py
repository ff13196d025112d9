"""Normalised residual rho = ||A X - I|| / (||A|| ||X|| eps) of correct inversions on the host engine,
the measurements behind utils/metrics.py RHO_PER_N (python bench/residual_ratio.py)."""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import mpi_jordan_crazy_acceleration_amd as gj
C = gj.load_native()
eps = {"fp64": 2.220446049250313e-16, "fp32": 1.1920928955078125e-07}
for dt in ["fp64", "fp32"]:
  for gen in ["random", "randshift", "absdiff", "hilbert"]:
    for n, m in [(100, 8), (300, 16), (600, 32), (1000, 64), (1500, 128)]:
        for seed in [1, 2]:
            eng = C.Engine(C.host_device(8), C.self_comm(), n, m, dt)
            eng.generate(gen, seed)
            st = eng.solve()
            if st["status"] != 0:
                print(dt, gen, n, m, seed, "status", st["status"]); continue
            na = eng.input_norm_inf(); ni = eng.result_norm_inf()
            r = eng.residual_generated(gen, seed)
            print(f"{dt} {gen:9s} n={n:5d} m={m:3d} seed={seed} res={r:.3e} |A|={na:.3e} |X|={ni:.3e} rho={r/(na*ni*eps[dt]):.3e} rho/n={r/(na*ni*eps[dt]*n):.3e}", flush=True)
