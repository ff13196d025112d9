"""Stream-ordered virtual ranks (AsyncLoopbackComm) on the CPU with real asynchronous streams
(AsyncHostDevice): the engine's MAIN / SIDE / COMM streams run on their own threads, collectives
never drain a stream, and random per-rank arrival delays reorder everything between runs.  A
missing event dependency shows up here as a wrong inverse (the synchronous transports hide it).
Reference semantics: the distributed Jordan() of main.cpp:953-1204 (MPI_Allreduce :1074,
MPI_Bcast :1097, MPI_Send/Recv :1118-1131)."""
import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix


def _inv(A, m, p, depth, jitter, chunk_cols=0, comm="async"):
    eng = gj.GaussJordan(block_size=m, ranks=p, device="cpu", comm=comm, depth=depth, jitter_us=jitter,
                         host_threads=1, chunk_cols=chunk_cols)
    rep = eng.run(A.shape[0], input=A, keep_inverse=True)
    assert rep["status"] == 0, rep["message"]
    return rep


@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("depth", [1, 3])
def test_async_ranks_match_numpy(p, depth):
    n, m = 150, 8
    A = generate_matrix(n, "random", 40 + p)[::-1].copy()  # off-diagonal pivots (row exchanges)
    rep = _inv(A, m, p, depth, jitter=300.0, chunk_cols=48)
    ref = np.linalg.inv(A)
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-10
    assert rep["stats"]["offdiag_pivots"] > 0
    assert rep["comm"].startswith("async-loopback") or p == 1
    assert rep["device"].startswith("host-async")


@pytest.mark.parametrize("depth", [2, 4])
def test_async_ranks_odd_chunk_tail(depth):
    """The chunk plan of n = 8192, m = 60 at p = 8 in miniature: 137 block rows, auto chunks of 68
    blocks and a one-block last chunk and panel (profiles/depth_pgt1.md, the depth-2 ordering item),
    jittered asynchronous ranks."""
    n, m = 137 * 8, 8
    A = generate_matrix(n, "random", 5)[::-1].copy()
    rep = _inv(A, m, 8, depth, jitter=300.0)
    ref = np.linalg.inv(A)
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-8


@pytest.mark.parametrize("p", [2, 4])
def test_async_equals_synchronous_loopback_bitwise(p):
    # same kernels, same operand order: the asynchronous schedule may only change timing
    n, m = 120, 6
    A = generate_matrix(n, "random", 7)
    sync = _inv(A, m, p, 2, 0.0, chunk_cols=36, comm="loopback")
    for seed_jitter in (50.0, 400.0):
        asy = _inv(A, m, p, 2, seed_jitter, chunk_cols=36)
        assert np.array_equal(asy["inverse"], sync["inverse"])


def test_async_direct_broadcast(monkeypatch):
    # the direct scatter + exchange broadcast's grouped point-to-point rounds, asynchronously
    monkeypatch.setenv("GJ_BCAST", "direct")
    monkeypatch.setenv("GJ_BCAST_MIN", "1")
    n, m = 130, 5
    A = generate_matrix(n, "random", 3)[::-1].copy()
    rep = _inv(A, m, 5, 2, 200.0, chunk_cols=40)
    ref = np.linalg.inv(A)
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-10


def test_async_singular_agreed_by_all_ranks():
    n, m = 60, 6
    A = generate_matrix(n, "random", 1)
    A[:, 7] = 0.0  # exactly singular
    eng = gj.GaussJordan(block_size=m, ranks=3, device="cpu", comm="async", jitter_us=100.0, host_threads=1)
    rep = eng.run(n, input=A)
    assert rep["status_name"] == "singular matrix"
