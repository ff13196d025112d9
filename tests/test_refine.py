"""fp32 made meaningful: the residual of an fp32 solve is checked in fp64 (fp64
A, widened inverse; reference main.cpp:490-507 is fp64), and A x = b is refined with the residual
in fp64: x_{k+1} = x_k + inv(A) (b - A x_k) (Engine::solve_rhs)."""
import os

import numpy as np
import pytest

from mpi_jordan_crazy_acceleration_amd import GaussJordan
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix


def _run(device, dtype, n, m, ranks=1, **extra):
    return GaussJordan(block_size=m, ranks=ranks, device=device, dtype=dtype, extra=extra).run(
        n, gen="random", seed=3, rhs="ones")


@pytest.mark.parametrize("ranks", [1, 3])
def test_fp32_refinement_reaches_fp64_accuracy(ranks):
    n, m = 240, 16
    r = _run("cpu", "fp32", n, m, ranks)
    assert r["status"] == 0
    h = r["axb_history"]
    assert h[0] > 1e-7  # x = inv32(A) b alone: fp32 accuracy
    assert r["refine_converged"] and r["axb_backward_error"] < 1e-15
    assert h[-1] < 1e-12 and all(b < a for a, b in zip(h, h[1:]))
    A = generate_matrix(n, "random", 3)
    x = np.linalg.solve(A, np.ones(n))
    # x itself: the refined solution matches the fp64 LAPACK solution to fp64 accuracy (times kappa)
    assert r["x_head"] is not None
    assert np.allclose(r["x_head"], x[: len(r["x_head"])], rtol=1e-9, atol=1e-12)


def test_fp32_residual_is_fp64():
    n, m = 200, 16
    r = _run("cpu", "fp32", n, m)
    assert r["residual_fp64"] is True
    A = generate_matrix(n, "random", 3)
    inv32 = np.linalg.inv(A.astype(np.float32).astype(np.float64))  # what an fp32 solve approximates
    ref = np.abs(A @ inv32 - np.eye(n)).sum(axis=1).max()
    # the reported residual is an fp64 quantity of order of the fp32 error, never 0 or fp32-noise-free
    assert 1e-8 < r["residual"] < 1e-1 and ref < 1e-1


def test_fp32_residual_falls_back_when_fp64_does_not_fit(monkeypatch):
    monkeypatch.setenv("GJ_TEST_ALLOC_FAIL", "0:residual64")
    r = _run("cpu", "fp32", 120, 8)
    assert r["status"] == 0 and r["residual_fp64"] is False


def test_fp64_rhs_converges_in_at_most_two_steps():
    r = _run("cpu", "fp64", 256, 32)
    assert r["refine_converged"] and r["refine_steps"] <= 2 and r["axb_backward_error"] < 1e-15


@pytest.mark.gpu
@pytest.mark.parametrize("n,m", [(4096, 128), (3000, 64)])
def test_gpu_fp32_refinement(n, m):
    r = _run("gpu", "fp32", n, m)
    assert r["status"] == 0 and r["residual_fp64"] is True
    assert r["refine_converged"], r["axb_history"]
    assert r["axb_history"][-1] < 1e-10


@pytest.mark.parametrize("n,m", [(12, 3), (16, 4)])
def test_diverging_refinement_returns_best_iterate(n, m):
    # an fp32 inverse of a Hilbert matrix (kappa ~ 1e16) makes refinement diverge; the
    # returned x and its residual must be the best iterate's, not the last one's
    r = GaussJordan(block_size=m, device="cpu", dtype="fp32").run(n, gen="hilbert", rhs="ones")
    assert r["status"] == 0 and not r["refine_converged"]
    h = r["axb_history"]
    assert len(h) >= 2 and h[-1] > h[0]
    assert r["axb_residual"] == pytest.approx(min(h), rel=1e-12)  # ||b||_inf = 1
    assert r["refine_steps"] == h.index(min(h))
