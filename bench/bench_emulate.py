#!/usr/bin/env python3
"""Per-rank critical-path emulation of a p-GPU solve on ONE GPU (ShadowComm, gj/comms.hpp).

Rank 0 of a p-rank job runs alone: 1/p of the rows, all pivot searches, panel pieces, chunk
pipeline and full-width trailing updates; peers' rows arrive as zeros.  Without --bw broadcasts are
local (the time is a LOWER bound of the real p-GPU step, xGMI transfer time excluded).  With
--bw GB/s every collective is replaced by its modelled cost (ShadowComm's CostModel: --lat us +
bytes / bw on --channels spin workgroups of an RCCL channel's footprint, competing with the
trailing update for CUs); "comm_hidden" is then the share of the modelled transfer time that the
look-ahead hid: 1 - (t_model - t_free) / modelled.  Not a headline number (see bench.py).

    python bench/bench_emulate.py --ranks 1 2 4 8 --size 32768 [--bw 100 --lat 20]
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
    ap.add_argument("--depth", type=int, nargs="+", default=[0], help="0 = the engine's auto choice")
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--chunk-cols", type=int, default=0)
    ap.add_argument("--bw", type=float, nargs="*", default=[],
                    help="cost-model bandwidths in GB/s (each also runs the comm-free baseline)")
    ap.add_argument("--lat", type=float, default=20.0, help="cost-model latency per collective, us")
    ap.add_argument("--channels", type=int, default=16, help="cost-model workgroups per collective")
    ap.add_argument("--bcast", choices=["ring", "direct", "both"], default="ring",
                    help="broadcast algorithm under the cost model (direct = scatter + slice exchange, "
                         "two point-to-point rounds over p-1 links)")
    args = ap.parse_args()
    import torch  # noqa: F401  (shares libamdhip64 with the extension)
    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    dev = C.hip_device(0)
    def run(p, d, bw, algo="ring"):
        os.environ["GJ_BCAST"] = algo
        comm = (C.shadow_comm(p, bw, args.lat if bw > 0 else 0.0, args.channels, direct=(algo == "direct"))
                if p > 1 else C.self_comm())
        eng = C.Engine(dev, comm, args.size, args.block, args.dtype, args.chunk_cols, 1e-15, False, d)
        times, modelled = [], 0.0
        for _ in range(args.reps + 1):
            if p > 1:
                C.shadow_reset(comm)
                m0 = C.shadow_modelled_us(comm)
            eng.generate("random", 7)
            dev.sync()
            t0 = time.perf_counter()
            st = eng.solve()
            dev.sync()
            times.append(time.perf_counter() - t0)
            if p > 1:
                modelled = (C.shadow_modelled_us(comm) - m0) * 1e-6
        rows, depth = eng.layout["rows"], eng.layout["depth"]
        del eng
        return min(times[1:]), st, (rows, depth), modelled

    for p in args.ranks:
        for d in args.depth:
            t_free, st, (rows, dd), _ = run(p, d, 0.0)
            gemm_flops = 2.0 * rows * args.size * args.size  # this rank's share of 2N^3
            print(json.dumps({"p": p, "depth": dd, "n": args.size, "m": args.block, "status": st["status"],
                              "seconds": round(t_free, 4),
                              "job_gflops_if_comm_free": round(2 * args.size ** 3 / t_free / 1e9, 1),
                              "rank_tflops": round(gemm_flops / t_free / 1e12, 2),
                              "host_wait_ms": round(st["host_wait_ms"], 1)}), flush=True)
            algos = ["ring", "direct"] if args.bcast == "both" else [args.bcast]
            for bw, algo in [(b, a) for b in (args.bw if p > 1 else []) for a in algos]:
                t, st, (rows, dd), modelled = run(p, d, bw, algo)
                hidden = 1.0 - (t - t_free) / modelled if modelled > 0 else None
                print(json.dumps({"p": p, "depth": dd, "n": args.size, "bcast": algo if p > 2 else "ring",
                                  "model_bw_gbs": bw, "model_lat_us": args.lat,
                                  "model_channels": args.channels, "status": st["status"],
                                  "seconds": round(t, 4),
                                  "job_gflops_cost_model": round(2 * args.size ** 3 / t / 1e9, 1),
                                  "modelled_comm_s": round(modelled, 4),
                                  "comm_hidden": None if hidden is None else round(hidden, 3)}), flush=True)


if __name__ == "__main__":
    main()
