"""Reference-compatible front end for the one-process-per-GPU deployment.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m mpi_jordan_crazy_acceleration_amd.cli \\
        [options] n m [file]

The ``mpirun -np p ./a.out n m [file]`` contract of the reference (main.cpp:65-93, solve()
:343-519) over ``torch.distributed``: one rank per process (RCCL on GPUs, gloo + the native host
executor with ``--device cpu``), every rank parsing only its own block rows of ``file``
(``DistributedGaussJordan.load_file``).  Rank 0 prints exactly what the reference prints: ``A`` and
its corner, ``glob_time: %.2f`` (max over ranks), ``inverse matrix:`` + blank line, the inverse's
corner, ``residual: %e`` (or ``p == 1!`` with ``--residual compat`` on one rank).  Exit codes:
0 ok, 1 usage, 2 any failure (cannot open / cannot read / singular matrix / not enough memory).
The in-process ``build/gj`` binary is the same contract with threads instead of processes.
``--comm-timeout S``: a rank waiting longer than S seconds on a peer fails (every rank, naming the
step, phase and collective).  ``--same-gpu``: rehearse the p-rank RCCL path with every rank on
GPU 0 (each rank its own RCCL host over loopback sockets; functional check, not a timing).
"""
from __future__ import annotations

import json
import os
import sys


def _usage(prog: str) -> int:
    print(f"usage:{prog} n m [<file>]", flush=True)
    return 1


def _atoi(s: str) -> int:
    # C atoi: optional sign + leading digits, 0 when there are none
    s = s.strip()
    i, sign = 0, 1
    if i < len(s) and s[i] in "+-":
        sign = -1 if s[i] == "-" else 1
        i += 1
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    return sign * int(s[i:j]) if j > i else 0


def _corner(c) -> str:
    return "".join("".join(f"{v:.2f}\t" for v in row) + "\n" for row in c)


def main(argv=None) -> int:
    import argparse

    argv = sys.argv[1:] if argv is None else argv
    prog = "gj"
    ap = argparse.ArgumentParser(add_help=False, allow_abbrev=False)
    ap.add_argument("pos", nargs="*")
    ap.add_argument("--device", choices=["auto", "gpu", "cpu"], default="auto")
    ap.add_argument("--dtype", choices=["fp64", "fp32"], default="fp64")
    ap.add_argument("--gen", choices=["absdiff", "hilbert", "random", "randshift", "identity"], default="absdiff")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--residual", choices=["always", "compat", "never"], default="always")
    ap.add_argument("--print-max", type=int, default=10)
    ap.add_argument("--eps", type=float, default=1e-15)
    ap.add_argument("--depth", type=int, default=0)
    ap.add_argument("--pivot", choices=["block-min-inv-norm", "partial"], default="block-min-inv-norm")
    ap.add_argument("--chunk-cols", type=int, default=0)
    ap.add_argument("--host-threads", type=int, default=0)
    ap.add_argument("--comm-timeout", type=float, default=600.0)
    ap.add_argument("--bcast", choices=["auto", "ring", "direct"], default=None)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--same-gpu", action="store_true")
    try:
        args, unknown = ap.parse_known_args(argv)
    except SystemExit:
        return _usage(prog)
    if unknown or not (2 <= len(args.pos) <= 3):
        return _usage(prog)
    n, m = _atoi(args.pos[0]), _atoi(args.pos[1])
    if n <= 0 or m <= 0 or args.print_max < 0:
        return _usage(prog)
    path = args.pos[2] if len(args.pos) == 3 else None
    if args.bcast:
        os.environ["GJ_BCAST"] = args.bcast

    from .runtime_env import configure_runtime_env

    configure_runtime_env()
    import torch
    import torch.distributed as dist

    from ._native import load_native
    from .parallel.dist import DistributedGaussJordan

    C = load_native()
    gpu = args.device == "gpu" or (args.device == "auto" and C.device_count() > 0)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_gpu:
        # rehearsal of the p-rank RCCL path on ONE GPU (as bench.py --same-gpu): every rank is its
        # own RCCL "host", so RCCL accepts the shared device and connects the ranks by sockets
        local = 0
        os.environ["NCCL_HOSTID"] = f"gj-cli-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    from datetime import timedelta

    pg_timeout = timedelta(seconds=max(60.0, args.comm_timeout))
    if gpu:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world,
                                timeout=pg_timeout)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout)
    out = (lambda s: print(s, end="", flush=True)) if rank == 0 else (lambda s: None)
    nm = min(n, args.print_max)
    try:
        try:
            solver = DistributedGaussJordan(n, m, dtype=args.dtype, chunk_cols=args.chunk_cols, eps=args.eps,
                                            host_threads=args.host_threads, depth=args.depth, pivot=args.pivot,
                                            local_rank=local if gpu else None, comm_timeout=args.comm_timeout)
        except C.GJError as e:  # agreed on every rank inside the constructor
            out("Not enough memory!\n" if e.status == 2 else f"error: {e}\n")
            return 2
        if path is not None:
            try:
                solver.load_file(path, args.host_threads)
            except FileNotFoundError:
                out(f"cannot open {path}\n")
                return 2
            except ValueError:
                out(f"cannot read {path}\n")
                return 2
        else:
            solver.generate(args.gen, args.seed)
        out("A\n" + _corner(solver.corner(nm, "input")))
        try:
            st = solver.solve()
        except C.GJError as e:
            if e.status != 6:  # not a communication failure
                raise
            # a peer died or hung: every rank names its step, phase and collective (Engine::solve)
            # and leaves at once -- tearing the process group down could block on the dead peer
            print(f"gj: rank {rank}: {e}", file=sys.stderr, flush=True)
            os._exit(2)
        if st["status"] != 0:
            out("singular matrix\n" if st["status"] == 1 else
                "not enough memory for block\n" if st["status"] == 7 else f"unknown error: {st['status']}\n")
            return 2
        t = torch.tensor([st["seconds"]], dtype=torch.float64, device="cuda" if gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        glob = float(t.item())
        out(f"glob_time: {glob:.2f}\ninverse matrix:\n\n" + _corner(solver.corner(nm, "result")))
        want_res = args.residual == "always" or (args.residual == "compat" and (world != 1 or args.gen == "hilbert"))
        res = None
        if want_res:
            if path is not None:
                try:
                    res = solver.residual_file(path, args.host_threads)
                except FileNotFoundError:
                    out(f"cannot open for residual {path}\n")
                    return 2
                except ValueError:
                    out(f"cannot read for residual {path}\n")
                    return 2
            else:
                res = solver.residual_generated(args.gen, args.seed)
            out(f"residual: {res:e}\n")
        elif args.residual == "compat":
            out("p == 1!\n")
        if args.json and rank == 0:
            print(json.dumps({"n": n, "m": m, "ranks": world, "device": "gpu" if gpu else "cpu",
                              "dtype": args.dtype, "status": st["status"], "glob_time": glob,
                              "gflops_nominal": 2.0 * n ** 3 / glob / 1e9 if glob > 0 else 0.0,
                              "residual": res, "offdiag_pivots": st["offdiag_pivots"]}),
                  file=sys.stderr, flush=True)
        return 0
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
