"""Multi-process distributed engine over torch.distributed/gloo (the CPU form of the RCCL path).

Each process is one rank (as under `mpirun -np p`, reference main.cpp:65-93); the native HostDevice
executes the same Engine protocol as a GPU rank, collectives trampoline into gloo."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, m, depth, kind, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd.parallel import DistributedGaussJordan
    from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gj = DistributedGaussJordan(n, m, depth=depth, host_threads=2)
        if kind == "file":
            A = generate_matrix(n, "random", 11)
            gj.load(A)
        else:
            gj.generate(kind, 0)
        st = gj.solve()
        inv = gj.gather_inverse()
        if kind == "file":
            res = gj.residual(A)
        else:
            res = gj.residual_generated(kind, 0)
        corner = gj.corner(4)
        q.put((rank, st["status"], res, inv, corner))
    finally:
        dist.destroy_process_group()


def _run(world, n, m, depth, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, m, depth, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda r: r[0])


@pytest.mark.parametrize("world,n,m,depth,kind", [
    (2, 37, 5, 1, "file"),
    (2, 64, 8, 3, "absdiff"),
    (3, 50, 6, 2, "file"),
])
def test_gloo_distributed_inverse(world, n, m, depth, kind):
    from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix

    out = _run(world, n, m, depth, kind)
    A = generate_matrix(n, "random", 11) if kind == "file" else generate_matrix(n, kind, 0)
    ref = np.linalg.inv(A)
    for rank, status, res, inv, corner in out:
        assert status == 0
        assert res < 1e-8, res
        assert out[0][2] == res  # residual is a collective: identical on every rank
        assert np.allclose(corner, ref[:4, :4], rtol=1e-8, atol=1e-10)
    inv = out[0][3]
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-9


def test_gloo_direct_bcast(monkeypatch):
    # the direct broadcast's two grouped point-to-point rounds over real processes (spawned ranks
    # inherit the environment): torch.distributed isend/irecv here, ncclSend/ncclRecv on xGMI
    from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix

    monkeypatch.setenv("GJ_BCAST", "direct")
    monkeypatch.setenv("GJ_BCAST_MIN", "1")
    n = 50
    out = _run(4, n, 6, 2, "file")
    ref = np.linalg.inv(generate_matrix(n, "random", 11))
    for rank, status, res, inv, corner in out:
        assert status == 0 and res < 1e-8, (status, res)
    assert np.abs(out[0][3] - ref).max() / np.abs(ref).max() < 1e-9
