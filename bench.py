#!/usr/bin/env python3
"""Headline benchmark: N = 32768 fp64 dense block Gauss-Jordan inversion on 1/2/4/8 MI355X.

Metric (BASELINE.json): "GFLOP/s + wall-clock, N=32768 dense Gauss-Jordan at 1/2/4/8 MI355X".
One *step* = one complete inversion of a fresh synthetic random dense N x N fp64 matrix
(uniform [-1, 1), seeded, generated on the GPUs inside the timed region) with the block-row-cyclic
native engine: look-ahead pivot search, chunk-pipelined RCCL pivot-row broadcast, MFMA elimination,
final row/column permutation into the reference's distribution.  GFLOP/s uses the nominal
inversion count 2 N^3 and is the whole-job aggregate (strong scaling: N fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]            # starts its own N rank processes
    torchrun --nproc-per-node N bench.py --gpus N --steps K ...    # or one rank per process from torchrun

Process model (the reference's SPMD start, main.cpp:65-74): one process per GPU.  Without
torchrun's environment, ``--gpus N > 1`` makes this process a launcher that never touches a GPU: it
starts N copies of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, forwards rank 0's
JSON line, stops the survivors when a rank fails, and exits with the largest child status.  The
ranks bootstrap over gloo (the two RCCL unique ids, the timing barrier, the per-rank statistics);
every collective of the solve is RCCL, issued by the native engine from C++.

Failure handling: every host wait of the engine is bounded by ``--comm-timeout`` (default 90 s,
below the driver's 600 s), so a hung peer turns into a non-zero exit on every rank, each naming
its step, phase and the collective it sat in.  A wrong inverse is a failure too: after the timed
loop the residual ||A A^-1 - I||_inf (the reference's check, main.cpp:490-507) is normalised by
||A|| ||A^-1|| eps and gated at 2n (``utils.metrics``, LAPACK's inverse test ratio); non-finite or
above the gate, the JSON line says ``"check": "residual_failed"`` and every rank exits 2.

``--same-gpu`` (rehearsal on a one-GPU box): all ranks share device 0 and RCCL is told that every
rank is its own host (``NCCL_HOSTID``), so it accepts the duplicate device and connects the ranks
through its network transport over loopback sockets.  This executes the multi-rank RCCL path
(RcclComm's groups, broadcasts, all-gathers, point-to-point exchange) on one GPU; the timing is not
an xGMI measurement.

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
ROOT = os.path.dirname(os.path.abspath(__file__))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults = the round driver's command (python3 bench.py --gpus 1 --steps 20 --warmup 5), so
    # every number quoted from a bare `python bench.py` is the sustained-load figure it records
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", dest="n", type=int, default=32768, help="matrix order N")
    ap.add_argument("--block", dest="m", type=int, default=128, help="pivot block size m")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--gen", default="random")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--chunk-cols", type=int, default=0)
    ap.add_argument("--depth", type=int, default=0,
                    help="elimination steps fused per trailing update (0 = the engine's choice)")
    ap.add_argument("--no-residual", action="store_true")
    ap.add_argument("--pivot", choices=["block-min-inv-norm", "partial"], default="block-min-inv-norm",
                    help="pivot rule: the reference's smallest ||inv(block)|| (the benchmarked algorithm) "
                         "or block partial pivoting (a faster alternative mode)")
    ap.add_argument("--force-rccl", action="store_true", help="use the RCCL communicator even at 1 rank")
    ap.add_argument("--bcast", choices=["auto", "ring", "direct"], default=None,
                    help="pivot-row broadcast at p > 2 (default: GJ_BCAST or auto = both timed at "
                         "engine setup, the faster kept)")
    ap.add_argument("--gemm-variant", default=None, help="big | narrow | squarepf | bigpf | glds | auto (tile for every launch; microbenchmarks)")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu = the native host executor with gloo collectives (rehearses the exact "
                         "multi-rank script on a machine without GPUs; not a performance mode)")
    ap.add_argument("--host-threads", type=int, default=1, help="host executor threads per rank (--device cpu)")
    ap.add_argument("--comm-timeout", type=float, default=90.0,
                    help="seconds a rank waits on a peer before it aborts the communicators and exits")
    ap.add_argument("--profile", action="store_true",
                    help="per-phase device timers; the JSON line carries the max over ranks")
    ap.add_argument("--rhs", choices=["ones", "random"], default=None,
                    help="time a SOLVE of A x = b: the inversion plus x = inv(A) b refined in fp64 against A "
                         "regenerated in fp64 (BASELINE config 5: --dtype fp32 --size 65536 --gen randshift "
                         "--rhs ones); the JSON line carries the refinement history")
    ap.add_argument("--refine", type=int, default=-1, help="refinement step budget (-1: 2 fp64 / 10 fp32)")
    ap.add_argument("--same-gpu", action="store_true",
                    help="rehearsal: every rank on device 0, RCCL over loopback sockets (see above)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher (no GPU)
def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv) -> int:
    """Start args.gpus rank processes of this script; never initialises a GPU itself."""
    import subprocess
    import threading

    n = args.gpus
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE, text=True, bufsize=1))

    def forward(r, p):
        for line in p.stdout:
            if r == 0:
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.write(f"[rank {r}] {line}")
                sys.stderr.flush()

    readers = [threading.Thread(target=forward, args=(r, p), daemon=True) for r, p in enumerate(procs)]
    for t in readers:
        t.start()
    # A failed rank: its peers exit on their own once their communication timeout expires; give
    # them that long (plus teardown), then stop whatever is left.
    grace = args.comm_timeout + 30.0
    deadline = None
    while any(p.poll() is None for p in procs):
        if deadline is None and any(p.returncode not in (None, 0) for p in procs):
            deadline = time.monotonic() + grace
        if deadline is not None and time.monotonic() > deadline:
            for r, p in enumerate(procs):
                if p.poll() is None:
                    sys.stderr.write(f"bench.py: rank {r} still running {grace:.0f} s after a peer failed; killed\n")
                    p.kill()
            break
        time.sleep(0.1)
    codes = []
    for p in procs:
        rc = p.wait()
        codes.append(rc if rc >= 0 else 128 - rc)
    for t in readers:
        t.join(timeout=5)
    if any(codes):
        sys.stderr.write(f"bench.py: rank exit codes {codes}\n")
    return max(codes)


_COMM_PHASE = {"pivot_rows": "row_bcast", "panel_pieces": "panel_pieces", "pivot_records": "pivot_exchange"}


def _comm_bandwidth(st):
    """Achieved bandwidth per collective kind of one rank's profiled solve."""
    out = {}
    phases = st.get("phases") or {}
    for kind, cb in (st.get("comm_bytes") or {}).items():
        ms = (phases.get(_COMM_PHASE[kind]) or {}).get("ms", 0.0)
        out[kind] = {"bytes": cb["bytes"], "calls": cb["calls"], "phase_ms": round(ms, 3),
                     "GB_s": round(cb["bytes"] / (ms * 1e6), 3) if ms > 0 else None}
    return out


def _merge_transports(per_rank):
    """RCCL channel connections per transport, summed over ranks (None: no RCCL in this run)."""
    if all(t is None for t in per_rank):
        return None
    out = {}
    for t in per_rank:
        for k, v in (t or {}).items():
            out[k] = out.get(k, 0) + v
    return out


# ----------------------------------------------------------------------------- one rank
def run_rank(args) -> int:
    gpu = args.device == "gpu"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.same_gpu:
        local = 0
        # RCCL refuses two ranks on one device of one host; as separate "hosts" they connect
        # through the socket transport (loopback).  Read by RCCL at communicator creation.
        os.environ["NCCL_HOSTID"] = f"gj-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")

    # Hardware queues and kernel-argument placement, before the first HIP call of the process
    # (mpi_jordan_crazy_acceleration_amd/runtime_env.py).
    sys.path.insert(0, ROOT)
    from mpi_jordan_crazy_acceleration_amd.runtime_env import configure_runtime_env

    configure_runtime_env()
    # which transport RCCL connects the ranks with (P2P over xGMI, or sockets): its INFO log of the
    # connection setup goes to a per-rank file, parsed after the warm-up (utils/rccl_log.py)
    rccl_log = None
    if gpu and (world > 1 or args.force_rccl):
        import tempfile

        from mpi_jordan_crazy_acceleration_amd.utils import rccl_log as _rl

        rccl_log = _rl.enable(os.path.join(tempfile.gettempdir(), f"gj_rccl_{os.getpid()}.log"))
    if args.bcast:
        os.environ["GJ_BCAST"] = args.bcast
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    if gpu:
        torch.cuda.set_device(local)
    if args.gemm_variant:
        C.set_gemm_variant(args.gemm_variant)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        # bootstrap only (ids, timing barrier, statistics); the solve's collectives are RCCL
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=timedelta(seconds=max(60.0, args.comm_timeout)))

    def fail(msg) -> int:
        # a failed rank leaves at once: its communicators may be aborted or hung on a dead peer,
        # and their teardown (or the bootstrap group's) must not decide the exit status
        print(f"bench.py: rank {rank}: {msg}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(2)

    comm_mode = {"one_comm": False, "hw_queues": None, "reason": ""}
    try:
        if not gpu:
            dev = C.host_device(args.host_threads)
            if world > 1:  # the GPU path's agreement, rehearsed (GJ_TEST_HW_QUEUES fakes a count)
                from mpi_jordan_crazy_acceleration_amd.parallel.dist import agree_comm_mode

                comm_mode = agree_comm_mode()
            if world > 1:
                from mpi_jordan_crazy_acceleration_amd.parallel.dist import TorchDistComm

                comm = C.py_comm(TorchDistComm(), rank, world)
            else:
                comm = C.self_comm()
        elif world > 1 or args.force_rccl:
            if world > 1:  # every rank takes the same communicator schedule, before any exists
                from mpi_jordan_crazy_acceleration_amd.parallel.dist import agree_comm_mode

                comm_mode = agree_comm_mode()
            ids = [[C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(ids, src=0)
            dev = C.hip_device(local)
            comm = C.rccl_comm(ids[0], world, rank, local, one_comm=comm_mode["one_comm"])
        else:
            dev = C.hip_device(local)
            comm = C.self_comm()
        # allocation is agreed on every rank inside the constructor (a rank that cannot allocate
        # makes every rank fail here, before any other collective)
        eng = C.Engine(dev, comm, args.n, args.m, args.dtype, args.chunk_cols, 1e-15, False, args.depth,
                       args.profile, args.comm_timeout, args.pivot)
    except RuntimeError as e:
        return fail(e)

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    rhs_b = None
    if args.rhs:
        import numpy as np

        rhs_b = (np.ones(args.n) if args.rhs == "ones" else
                 np.random.default_rng(args.seed + 1).uniform(-1.0, 1.0, args.n))
    rhs_info = {}

    def step():
        eng.generate(args.gen, args.seed)
        st = eng.solve()
        if rhs_b is not None and st["status"] == 0:  # the refined solve is part of the timed step
            _, info = eng.solve_rhs_generated(args.gen, args.seed, rhs_b, args.refine)
            rhs_info.clear()
            rhs_info.update(info)
        return st

    try:
        for _ in range(args.warmup):
            st = step()
            if st["status"] != 0:
                return fail(f"solve failed with status {st['status']}")
        if rccl_log:  # before the timed loop: every connection the solve uses is up after a warm-up
            from mpi_jordan_crazy_acceleration_amd.utils.rccl_log import transports

            print(f"bench.py: rank {rank}: RCCL transport {transports(rccl_log)}", file=sys.stderr, flush=True)
        barrier()
        t0 = time.perf_counter()
        stats = []
        step_ms = []  # wall time of every timed step (solve() returns after the device finished)
        for _ in range(args.steps):
            ts = time.perf_counter()
            stats.append(step())
            step_ms.append((time.perf_counter() - ts) * 1e3)
        barrier()
        t1 = time.perf_counter()
    except RuntimeError as e:
        return fail(e)
    st = stats[-1] if stats else {"status": 0, "offdiag_pivots": 0, "host_wait_ms": 0.0, "seconds": 0.0}
    # The gate checks the LAST TIMED solve (its output is still in the engine): the profiled solve
    # below runs another schedule, so a race of the unprofiled one must fail here.
    res = None
    norm_a = norm_inv = None
    if not args.no_residual and st["status"] == 0:
        try:
            norm_a = eng.input_norm_inf()
            norm_inv = eng.result_norm_inf()
            res = eng.residual_generated(args.gen, args.seed)
        except RuntimeError as e:
            return fail(e)
    try:
        # p > 1: one extra UNTIMED solve with the per-phase device timers, so a multi-GPU record
        # carries its own phase breakdown and host waits (the timed steps stay unprofiled)
        prof = None
        if world > 1 and not args.profile:
            eng.set_profile(True)
            prof = step()
            eng.set_profile(False)
            if prof["status"] != 0:
                return fail(f"profiled solve failed with status {prof['status']}")
    except RuntimeError as e:
        return fail(e)
    ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    mine = {
        "ms": ms,
        "step_ms": step_ms,
        "solve_s": [s["seconds"] for s in stats],
        "host_wait_ms": max([s["host_wait_ms"] for s in stats] or [0.0]),
        "phases": (prof or (stats[-1] if stats else {})).get("phases"),
        "profiled_solve_s": prof["seconds"] if prof else None,
        "profiled_host_wait_ms": prof["host_wait_ms"] if prof else None,
        "comm_bandwidth": _comm_bandwidth(prof) if prof else None,
        "policy": eng.policy,
        "rccl_transport": None,
    }
    if rccl_log:
        from mpi_jordan_crazy_acceleration_amd.utils.rccl_log import transports

        mine["rccl_transport"] = transports(rccl_log) or {}
    if dist.is_initialized():
        everyone = [None] * world
        dist.all_gather_object(everyone, mine)
    else:
        everyone = [mine]
    ms = max(e["ms"] for e in everyone)
    gflops = 2.0 * float(args.n) ** 3 / (ms / 1e3) / 1e9
    from mpi_jordan_crazy_acceleration_amd.utils.metrics import (RHO_PER_N, residual_bound, residual_ok,
                                                                  residual_ratio)

    bound = rho = None
    if args.no_residual:
        check = "skipped"
    else:
        bound = residual_bound(args.n, norm_a or 0.0, norm_inv or 0.0, args.dtype)
        bound = bound if bound == bound and bound != float("inf") else None  # strict JSON
        rho = residual_ratio(res, norm_a or 0.0, norm_inv or 0.0, args.dtype)
        check = "residual_ok" if residual_ok(res, args.n, norm_a or 0.0, norm_inv or 0.0, args.dtype) \
            else "residual_failed"
    if rank == 0:
        pol = dict(mine["policy"])
        solve_all = [x for e in everyone for x in e["solve_s"]]
        per_rank_max = [max(e["solve_s"] or [0.0]) for e in everyone]
        out = {
            "metric": "GFLOP/s + wall-clock, N=32768 dense Gauss-Jordan at 1/2/4/8 MI355X",
            "value": round(gflops, 3),
            "unit": "GFLOP/s (nominal 2N^3 per inversion, whole job)",
            "n_gpus": 1 if args.same_gpu else world,
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
                         + ("min-inverse-norm block pivoting)" if args.pivot == "block-min-inv-norm"
                            else "block partial pivoting)"),
                "global_batch": 1,
                "seq_len": args.n,
                "parallelism": (f"block-row-cyclic p={world} (" +
                                ("RCCL, ranks sharing one GPU over loopback sockets" if args.same_gpu else
                                 "RCCL over xGMI" if gpu else "gloo, host executor") + ")")
                               if world > 1 else ("single GPU" if gpu else "single host rank"),
                "n": args.n,
                "m": args.m,
                "depth": pol["depth"],
                "bcast": pol["bcast"],
            },
            "ranks": world,
            "comm": pol.pop("comm"),
            "comm_mode": comm_mode,
            "bcast_tuning": pol.pop("bcast_tuning"),
            "policy": pol,
            "solve_seconds_max": round(max(solve_all or [0.0]), 4),
            "solve_seconds_min": round(min(solve_all or [0.0]), 4),
            "rank_solve_seconds_max": [round(x, 4) for x in per_rank_max],
            # every timed step, max over ranks (wall ms incl. generation) -- the sustained-load drift
            "step_ms": [round(max(e["step_ms"][i] for e in everyone), 2) for i in range(args.steps)],
            "host_wait_ms_max": round(max(e["host_wait_ms"] for e in everyone), 3),
            "host_wait_ms": round(st["host_wait_ms"], 3),
            "rccl_transport": _merge_transports([e["rccl_transport"] for e in everyone]),
            "residual_inf": res,
            "residual_bound": bound,
            # normalised residual ||A X - I|| / (||A|| ||X|| eps), gated at RHO_PER_N * n
            "residual_ratio": (round(rho, 4) if rho is not None and rho != float("inf") else
                               (None if rho is None else "inf")),
            "residual_ratio_bound": RHO_PER_N * args.n,
            "norm_a_inf": norm_a,
            "norm_inv_inf": norm_inv,
            "check": check,
            "status": st["status"],
            "offdiag_pivots": st["offdiag_pivots"],
            "pivot_fallbacks": st.get("pivot_fallbacks", 0),
        }
        if args.same_gpu:
            out["same_gpu_rehearsal"] = True
        if rhs_b is not None:
            out["rhs"] = {
                "b": args.rhs,
                "timed": "generation + inversion (" + args.dtype + ") + x = inv(A) b refined in fp64",
                "refine_steps": rhs_info.get("steps"),
                "converged": rhs_info.get("converged"),
                "relative_residual_history": rhs_info.get("history"),
                "final_relative_residual": (rhs_info.get("history") or [None])[-1],
                "backward_error": rhs_info.get("backward_error"),
            }
        pols = [e["policy"] for e in everyone]
        if any({k: v for k, v in p.items() if k != "comm"} != {k: v for k, v in pols[0].items() if k != "comm"}
               for p in pols):
            out["policy_per_rank"] = [{k: v for k, v in p.items() if k not in ("comm", "bcast_tuning")}
                                      for p in pols]
        if args.profile or prof is not None:
            phases = {}
            for e in everyone:
                for name, v in (e["phases"] or {}).items():
                    phases[name] = max(phases.get(name, 0.0), round(v["ms"], 3))
            out["phases_ms_max"] = phases
        if prof is not None:
            out["comm_bandwidth"] = {
                "basis": "payload bytes of this rank's collectives of each kind / the device time of the "
                         "phase that issues them, in the untimed profiled solve (pivot_rows: row_bcast; "
                         "panel_pieces: panel_pieces, incl. the owner's piece GEMM; pivot_records: "
                         "pivot_exchange, incl. the argmin kernel) -- algorithm bandwidth, a lower bound on "
                         "the link rate",
                "per_rank": [e["comm_bandwidth"] for e in everyone],
            }
            out["profiled_solve"] = {
                "timed": False,
                "seconds_per_rank": [round(e["profiled_solve_s"], 4) for e in everyone],
                "host_wait_ms_per_rank": [round(e["profiled_host_wait_ms"], 3) for e in everyone],
            }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    if check == "residual_failed":
        print(f"bench.py: rank {rank}: residual {res} exceeds the bound {bound} (normalised {rho} > "
              f"{RHO_PER_N} n) for --gen {args.gen} N={args.n} {args.dtype}: wrong inverse",
              file=sys.stderr, flush=True)
        return 2
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
