"""File ingest for the one-process-per-GPU deployment (gloo + host executor on the CPU):
every rank maps the file and parses only its own block rows (reference read_matrix,
main.cpp:209-282, where one rank parses and sends), errors agreed on every rank, and the
torchrun CLI (`python -m mpi_jordan_crazy_acceleration_amd.cli n m [file]`) prints what the
in-process `gj` binary prints."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GJ = os.path.join(ROOT, "build", "gj")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(nproc, *args, timeout=180):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "--local-ranks-filter", "0",
           "-m", "mpi_jordan_crazy_acceleration_amd.cli", "--device", "cpu", *args]
    return subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout)


def _ref_lines(out):
    return [l for l in out.splitlines() if not l.startswith("[Gloo]") and not l.startswith("glob_time")]


@pytest.mark.parametrize("nproc,n,m", [(4, 61, 7), (3, 40, 5)])
def test_torchrun_cli_matches_gj(tmp_path, nproc, n, m):
    A = np.random.default_rng(5).uniform(-1, 1, (n, n)) + 3 * np.eye(n)
    f = tmp_path / "a.txt"
    np.savetxt(f, A, fmt="%.17g")
    r = _torchrun(nproc, str(n), str(m), str(f))
    assert r.returncode == 0, r.stderr[-3000:]
    g = subprocess.run([GJ, "--device", "cpu", "-p", str(nproc), str(n), str(m), str(f)],
                       capture_output=True, text=True, timeout=120)
    assert g.returncode == 0
    got, want = _ref_lines(r.stdout), _ref_lines(g.stdout)
    assert got[:-1] == want[:-1]  # A, corners, "inverse matrix:" (residual printed last)
    assert got[-1].startswith("residual: ") and float(got[-1].split()[1]) < 1e-12


def test_torchrun_cli_errors(tmp_path):
    r = _torchrun(2, "8", "2", str(tmp_path / "missing.txt"))
    assert r.returncode != 0 and "cannot open " in r.stdout
    bad = tmp_path / "bad.txt"
    bad.write_text(" ".join(["1"] * 40 + ["x"] + ["1"] * 30))  # rank 1's rows hold the bad token
    r = _torchrun(2, "8", "2", str(bad))
    assert r.returncode != 0 and "cannot read " + str(bad) in r.stdout
    r = _torchrun(2, "8")
    assert r.returncode != 0 and r.stdout.strip().endswith("usage:gj n m [<file>]")


def _worker(rank, world, port, path, n, m, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from mpi_jordan_crazy_acceleration_amd import load_native
    from mpi_jordan_crazy_acceleration_amd.parallel import DistributedGaussJordan
    from mpi_jordan_crazy_acceleration_amd.parallel.layout import global_rows

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C = load_native()
        rows = [int(r) for r in global_rows(n, m, world, rank)]
        with open("/proc/self/clear_refs", "w") as fh:  # reset the peak-RSS mark (VmHWM)
            fh.write("5")

        def hwm():
            for line in open("/proc/self/status"):
                if line.startswith("VmHWM"):
                    return int(line.split()[1]) * 1024
        h0 = hwm()
        part = C.read_matrix_rows(path, n, rows, 1)
        peak = hwm() - h0
        gj = DistributedGaussJordan(n, m, host_threads=1)
        gj.load_file(path, 1)
        st = gj.solve()
        res = gj.residual_file(path, 1)
        q.put((rank, rows, part, peak, st["status"], res))
    finally:
        dist.destroy_process_group()


def test_distributed_load_file_share_only(tmp_path):
    # n = 2400 fp64: 46 MB as a matrix, ~140 MB as text; 4 ranks -> ~11.5 MB share each
    n, m, world = 2400, 40, 4
    A = np.random.default_rng(9).uniform(-1, 1, (n, n)) + 4 * np.eye(n)
    f = tmp_path / "big.txt"
    np.savetxt(f, A, fmt="%.17g")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(f), n, m, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = n * n * 8
    for rank, rows, part, peak, status, res in out:
        assert np.array_equal(part, A[rows])
        # its share (~full/4) plus one 8 MiB text window, far below the matrix or the text
        assert peak < 0.75 * full, (rank, peak / 2**20)
        print(f"rank {rank}: peak RSS growth while reading {peak / 2**20:.1f} MiB (share {len(rows) * n * 8 / 2**20:.1f} MiB)")
        assert status == 0 and res < 1e-7


def test_torchrun_cli_hang_fails_fast():
    """`--comm-timeout`: a rank that never joins the pivot exchange of step 3 (GJ_TEST_HANG) makes
    the torchrun CLI job fail within the timeout, naming the step."""
    import time
    t0 = time.monotonic()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", GJ_TEST_HANG="1:3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "mpi_jordan_crazy_acceleration_amd.cli", "--device", "cpu", "--comm-timeout", "5", "64", "8"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    # the rank that waits in vain names the step; torchrun then stops the job (its peer may be
    # terminated before it prints: torchrun ends the other workers when one fails)
    assert "gj: rank 1: rank 1/2, step 3 of 8, phase pivot search: timed out after 5" in r.stderr, r.stderr[-3000:]
    assert time.monotonic() - t0 < 90
