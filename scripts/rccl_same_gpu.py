"""Probe: p RCCL ranks (processes) sharing ONE GPU, running the real asynchronous engine schedule.

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \
        scripts/rccl_same_gpu.py --size 2048 --block 128

Bootstrap over gloo (unique ids only); every rank drives cuda:0 through its own RcclComm.  Prints
one line per rank: residual, solve time and the broadcast choice.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", dest="n", type=int, default=2048)
    ap.add_argument("--block", dest="m", type=int, default=128)
    ap.add_argument("--gen", default="random")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))))
    import torch.distributed as dist
    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ids = [[C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else None]
    dist.broadcast_object_list(ids, src=0)
    dev = C.hip_device(0)
    comm = C.rccl_comm(ids[0], world, rank, 0)
    eng = C.Engine(dev, comm, args.n, args.m, "fp64", comm_timeout_s=60.0)
    for r in range(args.reps):
        eng.generate(args.gen, 11 + r)
        st = eng.solve()
        res = eng.residual_generated(args.gen, 11 + r)
        print(f"rank {rank}/{world} rep {r}: status {st['status']} residual {res:.3e} "
              f"solve {st['seconds']*1e3:.1f} ms offdiag {st['offdiag_pivots']} bcast {eng.layout['bcast']}",
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
