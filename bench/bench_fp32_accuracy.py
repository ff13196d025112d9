#!/usr/bin/env python3
"""What an fp32 inversion is worth at large N, one MI355X:

* the fp32 solve's residual ||A inv32 - I||_inf computed in fp64 (fp64 A regenerated, the inverse
  widened, fp64 MFMA accumulation), next to the fp64 solve's;
* A x = b (b = ones) with refinement x_{k+1} = x_k + inv32 (b - A x_k), the residual in fp64: the
  relative residual per step, and whether it converged (Engine::solve_rhs);
* the distance of the fp32 inverse from the fp64 one, max-row-sum relative: ||inv32 - inv64|| / ||inv64||.

    python bench/bench_fp32_accuracy.py --sizes 16384 32768 65536
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[16384, 32768])
    ap.add_argument("--block", type=int, default=128)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-distance", action="store_true")
    ap.add_argument("--gens", nargs="+", default=["random", "randshift"],
                    help="random: uniform[-1,1) (kappa ~ 1e7-1e9 at these n); randshift: + sqrt(n) I (well conditioned)")
    args = ap.parse_args()
    from mpi_jordan_crazy_acceleration_amd import GaussJordan, load_native
    import torch

    C = load_native()
    for n, gen in [(n, g) for n in args.sizes for g in args.gens]:
        out = {"n": n, "m": args.block, "gen": gen}
        for dt in ("fp32", "fp64"):
            t0 = time.perf_counter()
            r = GaussJordan(block_size=args.block, device="gpu", dtype=dt).run(
                n, gen=gen, seed=args.seed, rhs="ones")
            out[dt] = {"status": r["status"], "solve_s": round(r["glob_time"], 4),
                       "residual": r["residual"], "residual_fp64": r["residual_fp64"],
                       "axb_history": r["axb_history"], "refine_converged": r["refine_converged"],
                       "axb_backward_error": r["axb_backward_error"],
                       "wall_s": round(time.perf_counter() - t0, 1)}
            print(json.dumps({"n": n, "gen": gen, dt: out[dt]}), flush=True)
        if not args.no_distance:
            dev = C.hip_device(0)
            comm = C.self_comm()
            inv = {}
            for dt, tdt in (("fp64", torch.float64), ("fp32", torch.float32)):
                eng = C.Engine(dev, comm, n, args.block, dt)
                eng.generate(gen, args.seed)
                st = eng.solve()
                assert st["status"] == 0
                t = torch.empty((n, n), dtype=tdt, device="cuda")
                eng.download_rows_device(t.data_ptr(), n)
                inv[dt] = t
                del eng
            x64 = inv["fp64"]
            num = 0.0
            den = x64.abs().sum(dim=1).max().item()
            for r0 in range(0, n, 4096):  # row slabs: no n x n fp64 temporary
                d = inv["fp32"][r0:r0 + 4096].double() - x64[r0:r0 + 4096]
                num = max(num, d.abs().sum(dim=1).max().item())
            out["inv_distance_rel"] = num / den
            print(json.dumps({"n": n, "gen": gen, "inv_distance_rel": out["inv_distance_rel"], "inv64_norm": den}),
                  flush=True)
            del inv, x64
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
