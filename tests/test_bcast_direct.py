"""The direct broadcast (root scatter of 1/(p-1) slices + slice exchange, csrc/runtime/comm.cpp) and
its selection (GJ_BCAST / GJ_BCAST_MIN, Comm::tune_bcast).  On the CPU it runs over the loopback
communicator's grouped point-to-point path, the same code the RCCL communicator drives on xGMI, so
a slicing or matching error shows up as a wrong inverse here.  The reference has only MPI_Bcast
(main.cpp:1093-1097); parity of the result is the same as for the ring path."""
import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj


def _rand(n, seed):
    return np.random.default_rng(seed).standard_normal((n, n))


@pytest.mark.parametrize("p", [3, 4, 5, 8])
@pytest.mark.parametrize("n,m", [(37, 5), (64, 4), (10, 3)])
def test_direct_bcast_inverse_matches_numpy(monkeypatch, p, n, m):
    monkeypatch.setenv("GJ_BCAST", "direct")
    monkeypatch.setenv("GJ_BCAST_MIN", "1")  # every broadcast, even a few bytes, goes direct
    A = _rand(n, n * 7 + p)
    inv = gj.inverse(A, block_size=m, device="cpu", ranks=p)
    ref = np.linalg.inv(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-10


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_direct_bcast_bitwise_equal_to_ring(monkeypatch, depth):
    # a broadcast moves bytes: the algorithm must not change a single bit of the result
    n, m, p = 48, 4, 4
    A = np.eye(n)[::-1] + 0.01 * _rand(n, 5)  # off-diagonal pivots (row swaps)
    monkeypatch.setenv("GJ_BCAST", "ring")
    ring = gj.GaussJordan(block_size=m, ranks=p, device="cpu", depth=depth).inverse(A)
    monkeypatch.setenv("GJ_BCAST", "direct")
    monkeypatch.setenv("GJ_BCAST_MIN", "1")
    direct = gj.GaussJordan(block_size=m, ranks=p, device="cpu", depth=depth).inverse(A)
    assert np.array_equal(ring, direct)


def test_bcast_mode_is_validated(monkeypatch):
    monkeypatch.setenv("GJ_BCAST", "tree")
    with pytest.raises(Exception, match="GJ_BCAST"):
        gj.inverse(_rand(12, 0), block_size=3, device="cpu", ranks=3)


def test_auto_mode_stays_ring_off_gpu(monkeypatch):
    # auto only measures on a GPU transport; the host loopback keeps the transport's broadcast
    monkeypatch.delenv("GJ_BCAST", raising=False)
    C = gj.load_native()
    eng = C.Engine(C.host_device(2), C.self_comm(), 16, 4, "fp64")
    assert eng.layout["bcast"] == "ring"


def test_tune_bcast_binding_single_rank(monkeypatch):
    monkeypatch.setenv("GJ_BCAST", "auto")
    C = gj.load_native()
    comm = C.self_comm()
    assert comm.tune_bcast(C.host_device(1), 1 << 20) == "ring"
    assert comm.bcast_report() == "ring"


def test_engine_policy_knobs(monkeypatch):
    """The policy the engine reports follows its environment overrides (README "Runtime knobs"):
    the dense trailing-update build is on exactly where CUs are reserved (none on the host
    executor) unless GJ_DENSE_GEMM says otherwise; the look-ahead rows run on SIDE unless
    GJ_LA_SIDE=0."""
    C = gj.load_native()
    pol = C.Engine(C.host_device(1), C.self_comm(), 64, 8, "fp64").policy
    assert pol["dense_gemm"] is False and pol["reserve_cus"] == 0 and pol["look_ahead_rows"] == "SIDE"
    monkeypatch.setenv("GJ_DENSE_GEMM", "1")
    monkeypatch.setenv("GJ_LA_SIDE", "0")
    pol = C.Engine(C.host_device(1), C.self_comm(), 64, 8, "fp64").policy
    assert pol["dense_gemm"] is True and pol["look_ahead_rows"] == "COMM"
