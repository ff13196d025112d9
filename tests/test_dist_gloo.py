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


def _bits_worker(rank, world, port, n, m, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd.parallel import DistributedGaussJordan

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gj = DistributedGaussJordan(n, m, host_threads=1)
        gj.generate("random", 5)
        assert gj.solve()["status"] == 0
        inv = gj.gather_inverse()
        if rank == 0:
            np.save(out, inv)
    finally:
        dist.destroy_process_group()


def test_threaded_cli_and_process_ranks_same_bits(tmp_path, gj_bin):
    """The in-process threaded runner (`gj -p 8`, one host thread per rank: csrc/solver/runner.cpp,
    the same code path as `gj -p 8 --comm rccl` up to the transport) and one process per rank
    (torch.distributed, the bench / torchrun path) must produce the same inverse, bit for bit."""
    import subprocess

    n, m, p = 333, 12, 8
    binf = tmp_path / "inv.bin"
    r = subprocess.run([gj_bin, "--device", "cpu", "--comm", "loopback", "-p", str(p), "--host-threads", "1",
                        "--gen", "random", "--seed", "5", "--out", str(binf), str(n), str(m)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    threaded = np.fromfile(binf, dtype=np.float64).reshape(n, n)
    out = str(tmp_path / "proc.npy")
    mp.spawn(_bits_worker, args=(p, _free_port(), n, m, out), nprocs=p, join=True)
    procs = np.load(out)
    assert np.array_equal(threaded.view(np.int64), procs.view(np.int64))
