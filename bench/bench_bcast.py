#!/usr/bin/env python3
"""Ring (ncclBroadcast) vs direct (root scatter + slice exchange) pivot-row broadcast over xGMI, at
the message sizes the engine sends (m x chunk-width segments), through the engine's own RcclComm
(Comm::tune_bcast, csrc/runtime/comm.cpp).  One process per GPU, p > 2:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        bench/bench_bcast.py --mib 0.5 2 8 32

Rank 0 prints one JSON line per size with both timings (ms per broadcast, roots rotating) and the
choice the engine would make.  SURVEY.md §2.5 / §7.6 H5.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, nargs="+", default=[0.5, 2, 8, 32])
    args = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))))
    os.environ["GJ_BCAST"] = "auto"
    import torch
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd import load_native

    C = load_native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world < 3:
        print("bench_bcast.py: needs at least 3 ranks (at p <= 2 both algorithms are one send)", file=sys.stderr)
        return 2
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
    ids = [[C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else None]
    dist.broadcast_object_list(ids, src=0)
    dev = C.hip_device(local)
    comm = C.rccl_comm(ids[0], world, rank, local)
    os.environ["GJ_BCAST_MIN"] = "1"
    for mib in args.mib:
        nbytes = int(mib * (1 << 20))
        rep = comm.tune_bcast(dev, nbytes)
        if rank == 0:
            print(json.dumps({"p": world, "bytes": nbytes, "report": rep}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
