"""Consumption-point verification (GJ_VERIFY / SolveOptions::verify / `gj --verify`).

Every broadcast buffer is hashed on the stream that consumes it, right before the consumer, and the
hashes are compared with the root's after the solve (Engine::verify_hashes).  A read that happens
before its data arrived, or a corrupted copy, is then reported at its step, phase, buffer, root,
receiver and stream -- not only as a large final residual.  Reference: the blocking order of
MPI_Allreduce / MPI_Bcast / MPI_Send-Recv (main.cpp:1074-1131) that makes every step's inputs
complete by construction.  Runs on the CPU with truly asynchronous streams (AsyncHostDevice) and
jittered virtual ranks (AsyncLoopbackComm)."""
import os
import re
import subprocess

import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, m, p, depth=0, jitter=300.0, comm="async", **extra):
    eng = gj.GaussJordan(block_size=m, ranks=p, device="cpu", comm=comm, depth=depth, jitter_us=jitter,
                         host_threads=1, extra=dict(verify=True, **extra))
    return eng.run(n, gen="random", seed=3, keep_inverse=True)


@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("depth", [1, 2, 4])
def test_verify_clean_runs_pass(p, depth):
    rep = _run(200, 8, p, depth)
    assert rep["status"] == 0, rep["message"]
    A = generate_matrix(200, "random", 3)
    assert np.abs(A @ rep["inverse"] - np.eye(200)).sum(1).max() < 1e-9


def test_verify_clean_partial_pivoting_and_direct_bcast(monkeypatch):
    monkeypatch.setenv("GJ_BCAST", "direct")
    assert _run(180, 8, 4, 3, pivot="partial")["status"] == 0
    monkeypatch.setenv("GJ_HOST_FREE", "1")  # root-agnostic all-reduced pieces (p > 1 host-free chain)
    assert _run(180, 8, 4, 3)["status"] == 0


def _cli(env_extra, *args):
    env = dict(os.environ, GJ_VERIFY="1", **env_extra)
    return subprocess.run([os.path.join(ROOT, "build", "gj"), "--device", "cpu", "--comm", "async", "--jitter",
                           "300", *args], capture_output=True, text=True, timeout=180, env=env, cwd="/tmp")


def test_verify_reports_dropped_broadcast_wait_at_its_chunk():
    """GJ_TEST_DROP_WAIT=b removes MAIN's wait for a chunk's broadcast: with jittered ranks some rank
    updates with a stale chunk.  The hash mode names the first such chunk segment -- step, phase
    'trailing update', buffer Rb[..] chunk c segment j, its root and the receiver, stream MAIN."""
    r = _cli({"GJ_TEST_DROP_WAIT": "b"}, "-p", "4", "--gen", "random", "400", "16")
    assert r.returncode == 2, r.stdout + r.stderr
    m = re.search(r"GJ_VERIFY: step (\d+) \(panel \d+\), phase trailing update, buffer Rb\[\d\] chunk \d+ "
                  r"segment \d+, root rank (\d+): rank\(s\) \[([\d, ]+)\] consumed different bytes on stream MAIN",
                  r.stderr)
    assert m, r.stderr[-2000:]
    assert m.group(2) not in m.group(3).split(", ")  # the root itself never differs from itself


def test_verify_catches_corruption_at_its_step():
    """GJ_TEST_CORRUPT=1:9 zeroes rank 1's copy of step 9's normalised pivot row after its broadcast:
    reported at step 9 on rank 1, not only as the final residual."""
    r = _cli({"GJ_TEST_CORRUPT": "1:9"}, "-p", "4", "--gen", "random", "400", "16")
    assert r.returncode == 2, r.stdout + r.stderr
    assert re.search(r"GJ_VERIFY: step 9 \(panel \d+\), phase trailing update, buffer Rb\[\d\] chunk \d+ segment 1, "
                     r"root rank \d: rank\(s\) \[1\] consumed different bytes on stream MAIN", r.stderr), r.stderr


def test_verify_names_dropped_chunk_pass_wait_on_local_buffers():
    """GJ_TEST_DROP_WAIT=cp removes SIDE's wait for the chunk pass two panels back: SIDE then rewrites
    a panel's multiplier rows Lrow / H_t^T / pieces (rank-local, never broadcast) while COMM's chunk
    pass still reads them.  The rank-local hand-over hashes (producer SIDE at the panel's end, COMM
    before its first and after its last read) name the buffer, the step and the stream -- a class the
    broadcast hashes alone cannot see."""
    r = _cli({"GJ_TEST_DROP_WAIT": "cp"}, "-p", "1", "--gen", "random", "--depth", "2", "--chunk-cols", "16",
             "640", "8")
    assert r.returncode == 2, r.stdout + r.stderr
    assert re.search(r"GJ_VERIFY: step \d+ \(panel \d+\), phase chunk pass \(after its last read\), rank-local "
                     r"buffer (Lrow|Ht|panel pieces PP)\[\d\](\[\d\])?: rank\(s\) \[0\] saw different bytes on "
                     r"stream COMM than the SIDE stream left at the end of the panel \(rewritten while still being "
                     r"read", r.stderr), r.stderr[-2000:]


@pytest.mark.parametrize("drop", ["edit", "x"])
def test_verify_quiet_on_value_benign_drops(drop):
    """The other planted drops verify cannot and must not name (profiles/verify_r6.md): 'edit' is no
    hazard at run time (MAIN's wait for the owner edits is implied by its wait for each chunk's
    broadcast, tests/test_race_check.py), and under 'x' the chunk pass reads the next panel's columns
    of ITS OWN pivot rows, which the concurrent look-ahead update leaves unchanged (they are masked
    as zero rows) -- a memory-model race the happens-before checker reports, with identical bytes.
    No false alarm, correct inverse."""
    r = _cli({"GJ_TEST_DROP_WAIT": drop}, "-p", "3", "--gen", "random", "--check-residual", "1e-9", "400", "16")
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("p", [1, 3])
def test_verify_local_slots_clean_with_race_check(p):
    """The rank-local hash launches are themselves ordered: the happens-before checker finds no race
    with GJ_VERIFY on, and the verified run passes."""
    eng = gj.GaussJordan(block_size=12, ranks=p, device="cpu", comm="async", depth=3, jitter_us=100.0,
                         host_threads=1, race_check=True, extra=dict(verify=True))
    rep = eng.run(300, gen="random", seed=3)
    assert rep["status"] == 0, rep["message"]
    assert rep["race_count"] == 0, "\n".join(rep["races"])


def test_verify_flag_on_the_cli_and_clean_exit():
    r = subprocess.run([os.path.join(ROOT, "build", "gj"), "--device", "cpu", "-p", "3", "--verify", "--gen",
                        "random", "300", "12"], capture_output=True, text=True, timeout=180, cwd="/tmp")
    assert r.returncode == 0, r.stderr
    assert "residual:" in r.stdout


# ---------------------------------------------------------------- chain / deferred split (Engine::split_)
def _inv_split(split, n, m, p, depth, comm="async", jitter=200.0, monkeypatch=None, **extra):
    monkeypatch.setenv("GJ_SPLIT", str(int(split)))
    eng = gj.GaussJordan(block_size=m, ranks=p, device="cpu", comm=comm, depth=depth, jitter_us=jitter,
                         host_threads=2, extra=dict(verify=True, **extra))
    rep = eng.run(n, gen="random", seed=8, keep_inverse=True)
    assert rep["status"] == 0, rep["message"]
    return rep["inverse"]


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("p,depth", [(1, 2), (1, 4), (3, 3), (8, 2), (4, 1)])
def test_split_column_updates_bit_identical(p, depth, mode, monkeypatch):
    """The look-ahead and in-panel column updates of the rows already used as pivot rows leave the
    pivot chain (deferred to COMM: mode 1, to MAIN: mode 2): the inverse is bit-identical to the
    unsplit schedule, under jittered asynchronous ranks with consumption-point verification on."""
    n, m = 64 * 11, 64
    a = _inv_split(0, n, m, p, depth, monkeypatch=monkeypatch)
    b = _inv_split(mode, n, m, p, depth, monkeypatch=monkeypatch)
    assert np.array_equal(a, b)
    A = generate_matrix(n, "random", 8)
    from mpi_jordan_crazy_acceleration_amd.utils.metrics import residual_ok
    res = np.abs(A @ b - np.eye(n)).sum(1).max()
    assert residual_ok(res, n, np.abs(A).sum(1).max(), np.abs(b).sum(1).max()), res


@pytest.mark.parametrize("mode", [1, 2])
def test_split_with_partial_pivoting(mode, monkeypatch):
    n, m = 64 * 9, 64
    a = _inv_split(0, n, m, 3, 3, monkeypatch=monkeypatch, pivot="partial")
    b = _inv_split(mode, n, m, 3, 3, monkeypatch=monkeypatch, pivot="partial")
    assert np.array_equal(a, b)


def test_split_policy_reported_and_off_when_not_applicable(native, monkeypatch):
    def pol(m):
        eng = native.Engine(native.host_device(2), native.self_comm(), 600, m, "fp64")
        return eng.policy["split"]
    assert pol(64) == 0  # opt-in (profiles/split_r5.md)
    monkeypatch.setenv("GJ_SPLIT", "1")
    assert pol(64) == 1
    assert pol(60) == 0  # the GPU tiles need 64 | m
    monkeypatch.setenv("GJ_SPLIT", "2")
    assert pol(64) == 2
    monkeypatch.setenv("GJ_SPLIT", "3")
    with pytest.raises(Exception, match="GJ_SPLIT"):
        pol(64)
    monkeypatch.setenv("GJ_SPLIT", "0")
    assert native.Engine(native.host_device(2), native.self_comm(), 600, 64, "fp64").policy["lat_wide"] is False
    monkeypatch.setenv("GJ_LAT_GLDS", "1")
    assert native.Engine(native.host_device(2), native.self_comm(), 600, 64, "fp64").policy["lat_wide"] is True


@pytest.mark.parametrize("p,depth", [(1, 2), (3, 3), (8, 2)])
def test_skip_columns_bit_identical(p, depth, monkeypatch):
    """One launch around the skipped columns computes the same products as one launch per side."""
    n, m = 64 * 11, 64
    out = []
    for sk in ("0", "1"):
        monkeypatch.setenv("GJ_SKIP_COLS", sk)
        monkeypatch.setenv("GJ_CHUNK_SKIP", sk)
        eng = gj.GaussJordan(block_size=m, ranks=p, device="cpu", comm="async", depth=depth, jitter_us=200.0,
                             host_threads=2, chunk_cols=64 * 4, extra=dict(verify=True))
        rep = eng.run(n, gen="random", seed=8, keep_inverse=True)
        assert rep["status"] == 0, rep["message"]
        out.append(rep["inverse"])
    assert np.array_equal(out[0], out[1])
