"""`--pivot partial`: block partial pivoting as a faster alternative to the
reference's smallest-||inv(block)|| rule (main.cpp:1039-1066).  Each rank scores its candidates by
their largest-magnitude entry, inverts only its winner, and the ranks' invertible winners compete
(largest magnitude; ties -> larger rank, then smaller local row).  When every rank's winner is
singular the step falls back to the reference's full search."""
import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix


def _mat(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "rand":
        return rng.standard_normal((n, n))
    if kind == "perm":  # reversed-identity dominant: off-diagonal pivots
        return np.eye(n)[::-1] + 0.01 * rng.standard_normal((n, n))
    return generate_matrix(n, kind)


@pytest.mark.parametrize("n,m", [(12, 3), (10, 3), (37, 5), (64, 8), (10, 12)])
@pytest.mark.parametrize("p", [1, 2, 3])
@pytest.mark.parametrize("kind", ["rand", "perm"])
def test_partial_inverse_matches_numpy(n, m, p, kind):
    A = _mat(kind, n, n * 7 + m)
    rep = gj.GaussJordan(block_size=m, ranks=p, device="cpu", pivot="partial").run(n, input=A, keep_inverse=True)
    assert rep["status"] == 0
    ref = np.linalg.inv(A)
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-10


@pytest.mark.parametrize("p", [1, 2, 4])
def test_partial_picks_largest_magnitude_block(p):
    m, Nr = 2, 6
    n = m * Nr
    rng = np.random.default_rng(1)
    A = rng.uniform(-1, 1, (n, n)) + 3 * np.eye(n)
    A[3 * m + 1, 0] = 50.0  # block row 3 holds the column's largest entry, and is invertible
    rep = gj.GaussJordan(block_size=m, ranks=p, device="cpu", pivot="partial").run(n, input=A, keep_inverse=True)
    assert rep["status"] == 0 and rep["stats"]["pivots"][0] == 3
    assert rep["stats"]["pivot_fallbacks"] == 0
    # the reference rule picks by ||inv|| instead (the diagonal blocks are strongly dominant)
    ref = gj.GaussJordan(block_size=m, ranks=p, device="cpu").run(n, input=A, keep_inverse=True)
    assert ref["stats"]["pivots"][0] != 3
    assert np.allclose(rep["inverse"], ref["inverse"], rtol=1e-9, atol=1e-12)


def test_partial_falls_back_when_every_winner_is_singular():
    # |i - j|: the largest entries of a block column sit in the farthest block row, whose block
    # (entries c + di - dj) has rank 2 -> singular for m >= 3: the step takes the full search
    n, m = 24, 4
    rep = gj.GaussJordan(block_size=m, ranks=2, device="cpu", pivot="partial").run(n, gen="absdiff", keep_inverse=True)
    assert rep["status"] == 0 and rep["stats"]["pivot_fallbacks"] > 0
    A = generate_matrix(n, "absdiff")
    ref = np.linalg.inv(A)
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-9


def test_partial_singular_matrix_reported():
    A = _mat("rand", 20, 2)
    A[:, 5] = 0
    rep = gj.GaussJordan(block_size=4, ranks=2, device="cpu", pivot="partial").run(20, input=A)
    assert rep["status"] == 1


def test_partial_cli_flag(gj_bin):
    import subprocess
    out = subprocess.run([gj_bin, "--device", "cpu", "-p", "3", "--pivot", "partial", "--gen", "random", "--json",
                          "200", "16"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "residual:" in out.stdout
    bad = subprocess.run([gj_bin, "--pivot", "nope", "10", "2"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 1


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,p", [(2048, 128, 1), (1000, 64, 3), (3000, 128, 4), (640, 200, 2)])
def test_partial_on_gpu(n, m, p):
    A = _mat("rand", n, 5)[::-1].copy()
    rep = gj.GaussJordan(block_size=m, ranks=p, device="gpu", comm="async" if p > 1 else "auto",
                         pivot="partial").run(n, input=A, keep_inverse=True)
    assert rep["status"] == 0
    ref = np.linalg.inv(A)
    # largest-entry block pivoting bounds ||inv(pivot block)|| less tightly than the reference rule:
    # 1e-8 relative at n = 3000 here (the reference rule: 1e-12), 6e-2 residual at N = 32768
    assert np.abs(rep["inverse"] - ref).max() / np.abs(ref).max() < 1e-6


@pytest.mark.gpu
def test_partial_fallback_on_gpu():
    rep = gj.GaussJordan(block_size=64, ranks=2, device="gpu", comm="async", pivot="partial").run(1024, gen="absdiff")
    assert rep["status"] == 0 and rep["stats"]["pivot_fallbacks"] > 0 and rep["residual"] < 1e-6


@pytest.mark.parametrize("p", [1, 2])
def test_partial_growth_guard(p):
    """A candidate with the column's largest entries but nearly singular (growth estimate
    ||inv(W)||_inf max|W| ~ 1e11, above the default bound 1e8) must not be accepted by partial
    pivoting: with the guard the step takes another rank's block or the full search; without it
    (pivot_growth = 0) the near-singular pivot is taken (a silently low-accuracy inverse)."""
    m, Nr = 4, 8
    n = m * Nr
    rng = np.random.default_rng(3)
    A = rng.uniform(-1, 1, (n, n)) + 2 * np.eye(n)
    u, v = rng.uniform(0.5, 1, m), rng.uniform(0.5, 1, m)
    A[2 * m:3 * m, :m] = 100.0 * np.outer(u, v) + 1e-9 * np.eye(m)  # block row 2: big, rank 1 + 1e-9 I
    guarded = gj.GaussJordan(block_size=m, ranks=p, device="cpu", pivot="partial").run(n, input=A, keep_inverse=True)
    assert guarded["status"] == 0 and guarded["stats"]["pivots"][0] != 2
    off = gj.GaussJordan(block_size=m, ranks=p, device="cpu", pivot="partial", extra={"pivot_growth": 0.0}).run(
        n, input=A, keep_inverse=True)
    assert off["status"] == 0 and off["stats"]["pivots"][0] == 2
    ref = np.linalg.inv(A)
    err = lambda r: np.abs(r["inverse"] - ref).max() / np.abs(ref).max()  # noqa: E731
    assert err(guarded) < 1e-10 and err(guarded) < err(off)
