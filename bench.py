#!/usr/bin/env python3
"""Headline benchmark: N = 32768 fp64 dense block Gauss-Jordan inversion on 1/2/4/8 MI355X.

Metric (BASELINE.json): "GFLOP/s + wall-clock, N=32768 dense Gauss-Jordan at 1/2/4/8 MI355X".
One *step* = one complete inversion of a fresh synthetic random dense N x N fp64 matrix
(uniform [-1, 1), seeded, generated on the GPUs inside the timed region) with the block-row-cyclic
native engine: look-ahead pivot search, chunk-pipelined RCCL pivot-row broadcast, MFMA elimination,
final row/column permutation into the reference's distribution.  GFLOP/s uses the nominal
inversion count 2 N^3 and is the whole-job aggregate (strong scaling: N fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]            # N = 1
    torchrun --nproc-per-node N bench.py --gpus N --steps K ...    # N > 1 (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  vs_baseline divides by the reference's own measured rate (30.8 GFLOP/s
nominal, its best published-in-survey run: N=8192, p=8 MPI ranks, SURVEY.md §7.5 — the reference
has no GPU path and no published N=32768 number).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REFERENCE_GFLOPS = 30.8  # reference N=8192 p=8 (35.73 s) -> 2N^3/t


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", dest="n", type=int, default=32768, help="matrix order N")
    ap.add_argument("--block", dest="m", type=int, default=128, help="pivot block size m")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--gen", default="random")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--chunk-cols", type=int, default=0)
    ap.add_argument("--depth", type=int, default=0,
                    help="elimination steps fused per trailing update (0 = the engine's choice: 2 up to "
                         "N=8192, else 4, profiles/small_n_sweep.md)")
    ap.add_argument("--no-residual", action="store_true")
    ap.add_argument("--force-rccl", action="store_true", help="use the RCCL communicator even at 1 rank")
    ap.add_argument("--bcast", choices=["auto", "ring", "direct"], default=None,
                    help="pivot-row broadcast at p > 2 (default: GJ_BCAST or auto = both timed at "
                         "engine setup, the faster kept)")
    ap.add_argument("--gemm-variant", default=None, help="big | narrow | tall (kernel tile config)")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu = the native host executor with gloo collectives (rehearses the exact "
                         "multi-rank script on a machine without GPUs; not a performance mode)")
    ap.add_argument("--host-threads", type=int, default=1, help="host executor threads per rank (--device cpu)")
    args = ap.parse_args()
    gpu = args.device == "gpu"

    # Hardware queues and kernel-argument placement, before the first HIP call of the process
    # (mpi_jordan_crazy_acceleration_amd/runtime_env.py: one queue per stream, so the two RCCL
    # communicators' kernels never queue behind each other; device-memory kernel arguments).
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mpi_jordan_crazy_acceleration_amd.runtime_env import configure_runtime_env

    configure_runtime_env()
    if args.bcast:
        os.environ["GJ_BCAST"] = args.bcast
    import torch
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if gpu:
        torch.cuda.set_device(local)
    if args.gemm_variant:
        C.set_gemm_variant(args.gemm_variant)
    if not gpu:
        dev = C.host_device(args.host_threads)
        if world > 1:
            from mpi_jordan_crazy_acceleration_amd.parallel.dist import TorchDistComm

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("gloo", rank=rank, world_size=world)
            comm = C.py_comm(TorchDistComm(), rank, world)
        else:
            comm = C.self_comm()
    elif world > 1 or args.force_rccl:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
        ids = [[C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        dev = C.hip_device(local)
        comm = C.rccl_comm(ids[0], world, rank, local)
    else:
        dev = C.hip_device(local)
        comm = C.self_comm()
    try:
        # allocation is agreed on every rank inside the constructor (a rank that cannot allocate
        # makes every rank fail here, before any other collective)
        eng = C.Engine(dev, comm, args.n, args.m, args.dtype, args.chunk_cols, 1e-15, False, args.depth)
    except RuntimeError as e:
        print(f"bench.py: rank {rank}: {e}", file=sys.stderr, flush=True)
        return 2

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    def step():
        eng.generate(args.gen, args.seed)
        return eng.solve()

    for _ in range(args.warmup):
        st = step()
        if st["status"] != 0:
            print(f"bench.py: rank {rank}: solve failed with status {st['status']}", file=sys.stderr)
            return 2
    barrier()
    t0 = time.perf_counter()
    inner = []
    for _ in range(args.steps):
        st = step()
        inner.append(st["seconds"])
    barrier()
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    if dist.is_initialized():
        t = torch.tensor([ms, max(inner)], dtype=torch.float64, device="cuda" if gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, inner_max = float(t[0]), float(t[1])
    else:
        inner_max = max(inner)
    res = None
    if not args.no_residual and st["status"] == 0:
        res = eng.residual_generated(args.gen, args.seed)
    gflops = 2.0 * float(args.n) ** 3 / (ms / 1e3) / 1e9
    if rank == 0:
        out = {
            "metric": "GFLOP/s + wall-clock, N=32768 dense Gauss-Jordan at 1/2/4/8 MI355X",
            "value": round(gflops, 3),
            "unit": "GFLOP/s (nominal 2N^3 per inversion, whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(gflops / REFERENCE_GFLOPS, 2),
            "dtype": args.dtype,
            "data": "synthetic: seeded uniform[-1,1) dense random matrix generated on-"
                    + ("GPU" if gpu else "host (--device cpu rehearsal)") + " each step",
            "config": {
                "model": f"dense block Gauss-Jordan inversion N={args.n} (block m={args.m}, in-place, "
                         "min-inverse-norm block pivoting)",
                "global_batch": 1,
                "seq_len": args.n,
                "parallelism": (f"block-row-cyclic p={world} (" + ("RCCL over xGMI" if gpu else "gloo, host executor")
                                + ")") if world > 1 else ("single GPU" if gpu else "single host rank"),
                "n": args.n,
                "m": args.m,
                "depth": eng.layout["depth"],
                "bcast": eng.layout["bcast"],
            },
            "bcast_tuning": comm.bcast_report(),
            "solve_seconds_max": round(inner_max, 4),
            "residual_inf": res,
            "status": st["status"],
            "offdiag_pivots": st["offdiag_pivots"],
            "host_wait_ms": round(st["host_wait_ms"], 3),
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
