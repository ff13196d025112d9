#!/usr/bin/env python3
"""Per-rank critical-path emulation of a p-GPU solve on ONE GPU (ShadowComm, gj/comms.hpp).

Rank 0 of a p-rank job runs alone: 1/p of the rows, all pivot searches, panel pieces, chunk
pipeline and full-width trailing updates; peers' rows arrive as zeros and broadcasts are local, so
the time is a LOWER bound of the real p-GPU step (xGMI transfer time excluded) and an UPPER bound
check of whether the look-ahead hides the pivot path.  Not a headline number (see bench.py).

    python bench/bench_emulate.py --ranks 1 2 4 8 --size 32768
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--block", type=int, default=128)
    ap.add_argument("--depth", type=int, nargs="+", default=[4])
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--chunk-cols", type=int, default=0)
    args = ap.parse_args()
    import torch  # noqa: F401  (shares libamdhip64 with the extension)
    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    dev = C.hip_device(0)
    for p in args.ranks:
        for d in args.depth:
            comm = C.shadow_comm(p) if p > 1 else C.self_comm()
            eng = C.Engine(dev, comm, args.size, args.block, args.dtype, args.chunk_cols, 1e-15, False, d)
            times = []
            for _ in range(args.reps + 1):
                if p > 1:
                    C.shadow_reset(comm)
                eng.generate("random", 7)
                dev.sync()
                t0 = time.perf_counter()
                st = eng.solve()
                dev.sync()
                times.append(time.perf_counter() - t0)
            t = min(times[1:])
            rows = eng.layout["rows"]
            gemm_flops = 2.0 * rows * args.size * args.size  # this rank's share of 2N^3
            print(json.dumps({"p": p, "depth": d, "n": args.size, "m": args.block, "status": st["status"],
                              "seconds": round(t, 4), "job_gflops_if_comm_free": round(2 * args.size ** 3 / t / 1e9, 1),
                              "rank_tflops": round(gemm_flops / t / 1e12, 2),
                              "host_wait_ms": round(st["host_wait_ms"], 1)}), flush=True)
            del eng


if __name__ == "__main__":
    main()
