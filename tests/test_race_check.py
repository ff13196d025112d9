"""Happens-before schedule checker (csrc/runtime/race_check.cpp).

The reference is race-free by construction: every step is a blocking MPI sequence
(main.cpp:1074 MPI_Allreduce, :1097 MPI_Bcast, :1118-1131 Send/Recv).  The engine's three streams,
events, stream-ordered collectives and host polling replace that; RaceCheckDevice derives
happens-before from the enqueue order (vector clocks per stream and host) and reports every pair
of conflicting accesses with no edge between them -- independent of timing, so a missing edge is
found on every run, not when a jittered run happens to expose it.

Covered here: the exact region geometry against brute force; the schedule matrix (p 1-8, depth
1-8, ring and direct broadcast, the one-block tail chunk of n = 8192 / m = 60 / p = 8 in miniature,
--pivot partial, both in-process transports) must be race-free; planted hazards (one ordering edge
left out under GJ_TEST_DROP_WAIT) must be reported with the buffer, both streams and the phases.
"""
import subprocess

import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd._native import load_native


def _brute(r):
    base, pitch, width, height = r
    s = set()
    for i in range(height):
        s.update(range(base + i * pitch, base + i * pitch + width))
    return s


def test_region_geometry_matches_brute_force():
    C = load_native()
    rng = np.random.default_rng(0)
    for _ in range(4000):
        regs = []
        for _ in range(2):
            pitch = int(rng.integers(1, 24))
            width = int(rng.integers(0, pitch + 1)) if rng.random() < 0.8 else int(rng.integers(0, 3 * pitch + 1))
            height = int(rng.integers(0, 6))
            base = 1000 + int(rng.integers(0, 60))
            if rng.random() < 0.3 and regs:  # same pitch as the other region (the fast path)
                pitch = regs[0][1]
                width = int(rng.integers(0, pitch + 1))
            regs.append((base, pitch, width, height))
        a, b = regs
        sa, sb = _brute(a), _brute(b)
        assert C._regions_overlap(a, b) == bool(sa & sb), (a, b)
        if C._region_covers(a, b):  # covering may be conservative (false), never wrong (true)
            assert sb <= sa, (a, b)
    # the cases the checker relies on being exact: column blocks of one row-major panel
    n8 = 600 * 8
    left = (0, n8, 40 * 8, 200)
    right = (40 * 8, n8, 40 * 8, 200)
    assert not C._regions_overlap(left, right)
    assert C._regions_overlap(left, (39 * 8, n8, 8, 200))
    assert C._region_covers((0, n8, 80 * 8, 200), right)


def _run(n, m, p, comm="async", ok=True, **kw):
    rep = gj.GaussJordan(block_size=m, ranks=p, device="cpu", comm=comm, race_check=True, host_threads=1,
                         **kw).run(n, gen="random", seed=3)
    if ok:
        assert rep["status"] == 0, rep["message"]
    return rep


@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("depth", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("bcast", ["ring", "direct"])
def test_schedule_matrix_race_free(p, depth, bcast, monkeypatch):
    monkeypatch.setenv("GJ_BCAST", bcast)
    monkeypatch.setenv("GJ_BCAST_MIN", "1")
    rep = _run(420, 20, p, depth=depth, chunk_cols=120)
    assert rep["race_ops"] > 0
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    assert rep["residual"] < 1e-8


@pytest.mark.parametrize("depth", [2, 4])
@pytest.mark.parametrize("bcast", ["ring", "direct"])
def test_one_block_tail_chunk_p8_race_free(depth, bcast, monkeypatch):
    # n = 8192, m = 60, p = 8 at the GPU failure (profiles/depth_pgt1.md): Nr = 137 blocks, chunks of
    # 68 blocks -> [0, 68), [68, 136), [136, 137); here m = 20 (the fused candidate-inverse +
    # selection path, 16 < m <= 128) with the same block counts and chunk plan
    monkeypatch.setenv("GJ_BCAST", bcast)
    monkeypatch.setenv("GJ_BCAST_MIN", "1")
    rep = _run(137 * 20 - 7, 20, 8, depth=depth, chunk_cols=68 * 20, jitter_us=30.0)
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    assert rep["residual"] < 1e-7


@pytest.mark.parametrize("p", [1, 3])
def test_partial_pivot_and_sync_transport_race_free(p):
    assert _run(300, 20, p, pivot="partial", depth=3)["race_count"] == 0
    if p > 1:
        rep = _run(300, 20, p, comm="loopback", depth=2)
        assert rep["race_count"] == 0, "\n".join(rep["races"])


@pytest.mark.parametrize("drop,buffer", [
    ("cp", "Ht["),       # SIDE rewrites a panel's H / Lrow / pieces while COMM's chunk pass of panel v-2 reads them
    ("b", "Rb["),        # MAIN's trailing update reads a chunk before its broadcast
    ("x", "X@"),         # the chunk pass reads the next panel's columns that the look-ahead update rewrites
    ("bcast_root", ""),  # cross-rank: receivers copy before the root's data is ready
])
def test_planted_hazard_is_reported(drop, buffer, monkeypatch):
    monkeypatch.setenv("GJ_TEST_DROP_WAIT", drop)
    # the asynchronous executor really runs the broken schedule: the inverse may come out wrong (or
    # "singular"); the report must be there either way
    rep = _run(300, 20, 3, ok=False, depth=2, chunk_cols=100)
    assert rep["race_count"] > 0
    text = "\n".join(rep["races"])
    assert buffer in text, text
    assert "no happens-before edge" in text and "rank " in text and "step " in text


def test_redundant_edge_is_not_reported(monkeypatch):
    # MAIN's wait for the owner edits is implied by its wait for each chunk's broadcast (the chunk
    # pass waits for the last panel piece, which follows every edit on SIDE): no report
    monkeypatch.setenv("GJ_TEST_DROP_WAIT", "edit")
    assert _run(300, 20, 3, depth=2, chunk_cols=100)["race_count"] == 0


def test_cli_race_check(gj_bin):
    r = subprocess.run([gj_bin, "--device", "cpu", "--comm", "async", "-p", "2", "--race-check", "--gen",
                        "random", "200", "20"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "race check: 0 unordered" in r.stderr
    env = dict(__import__("os").environ, GJ_TEST_DROP_WAIT="b")
    r = subprocess.run([gj_bin, "--device", "cpu", "--comm", "async", "-p", "2", "--race-check", "--gen",
                        "random", "200", "20"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2
    assert "race: unordered" in r.stderr


@pytest.mark.parametrize("p", [2, 3, 8])
@pytest.mark.parametrize("depth", [1, 2, 4])
def test_host_free_chain_multi_rank(p, depth, monkeypatch):
    """GJ_HOST_FREE=1 at p > 1: a panel's pivot chain is enqueued without a host wait per step, the
    owner-side launches read the pivot on the device and the panel piece travels by an all-reduce
    sum (non-owners contribute zeros).  Race-free, and bit-identical to the host-driven schedule."""
    ref = gj.GaussJordan(block_size=20, ranks=p, device="cpu", comm="async", depth=depth,
                         host_threads=1).run(420, gen="random", seed=3, keep_inverse=True)
    monkeypatch.setenv("GJ_HOST_FREE", "1")
    rep = _run(420, 20, p, depth=depth, jitter_us=20.0)
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    got = gj.GaussJordan(block_size=20, ranks=p, device="cpu", comm="async", depth=depth,
                         host_threads=1).run(420, gen="random", seed=3, keep_inverse=True)
    assert np.array_equal(got["inverse"], ref["inverse"])


@pytest.mark.parametrize("p", [1, 3])
@pytest.mark.parametrize("depth", [2, 4])
def test_look_ahead_rows_on_comm_race_free(p, depth, monkeypatch):
    """GJ_LA_SIDE=0 (the round-3 one-rank schedule: look-ahead rows on COMM, behind the previous
    panel's chunk pass) stays a supported knob: race-free and correct."""
    monkeypatch.setenv("GJ_LA_SIDE", "0")
    rep = _run(420, 20, p, depth=depth, chunk_cols=120)
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    assert rep["residual"] < 1e-8


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("p,depth,la_side", [(1, 2, "1"), (1, 4, "1"), (3, 2, "1"), (8, 2, "1"), (3, 4, "0")])
def test_split_column_updates_race_free(mode, p, depth, la_side, monkeypatch):
    """GJ_SPLIT=1/2 (the used rows' column updates deferred to COMM / MAIN): every deferred product
    is ordered against the chain's and the trailing update's accesses of the same rows."""
    monkeypatch.setenv("GJ_SPLIT", str(mode))
    monkeypatch.setenv("GJ_LA_SIDE", la_side)
    rep = _run(64 * 11, 64, p, depth=depth, chunk_cols=64 * 3, jitter_us=20.0)
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    assert rep["residual"] < 1e-8


@pytest.mark.parametrize("p,depth", [(1, 2), (1, 4), (3, 2), (8, 2), (4, 3)])
@pytest.mark.parametrize("skip", ["0", "1"])
def test_skip_columns_race_free(p, depth, skip, monkeypatch):
    """GJ_SKIP_COLS / GJ_CHUNK_SKIP: MAIN's chunk update and the chunk pass's normalisation as one
    launch around the look-ahead / panel columns (GemmExtra::skip_c0/c1) or one launch per side:
    race-free either way, and the same inverse."""
    monkeypatch.setenv("GJ_SKIP_COLS", skip)
    monkeypatch.setenv("GJ_CHUNK_SKIP", skip)
    rep = _run(64 * 11, 64, p, depth=depth, chunk_cols=64 * 4, jitter_us=20.0)
    assert rep["race_count"] == 0, "\n".join(rep["races"])
    assert rep["residual"] < 1e-8
