"""The residual when the whole inverse does not fit on some rank (p > 1): the reference's ring
(matrix_mult_matrix, main.cpp:534-642) as p strip broadcasts — agreed on every rank, same value as
the gathered path up to summation order, fp32 solves still checked in fp64."""
import pytest

from mpi_jordan_crazy_acceleration_amd import GaussJordan


def _run(monkeypatch, spec, dtype="fp64", ranks=3, n=150, m=8):
    if spec:
        monkeypatch.setenv("GJ_TEST_ALLOC_FAIL", spec)
    else:
        monkeypatch.delenv("GJ_TEST_ALLOC_FAIL", raising=False)
    return GaussJordan(block_size=m, ranks=ranks, device="cpu", dtype=dtype).run(n, gen="random", seed=4)


@pytest.mark.parametrize("dtype,ranks", [("fp64", 3), ("fp32", 4), ("fp64", 2)])
def test_streamed_residual_matches_gathered(monkeypatch, dtype, ranks):
    full = _run(monkeypatch, "", dtype, ranks)
    streamed = _run(monkeypatch, "1:residual", dtype, ranks)  # rank 1 cannot hold the inverse
    assert full["status"] == 0 and streamed["status"] == 0
    assert streamed["residual_fp64"] is True
    # the residual is itself rounding noise (~1e-10): only its magnitude is order-independent
    assert abs(streamed["residual"] - full["residual"]) <= 0.05 * full["residual"]


def test_residual_memory_failure_agreed(monkeypatch):
    r = _run(monkeypatch, "1:residual,2:residual_stream")
    assert r["status"] == 2  # NoMemory on every rank, no hang


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_streamed_residual_on_gpu_ranks(monkeypatch, dtype):
    def run(spec):
        if spec:
            monkeypatch.setenv("GJ_TEST_ALLOC_FAIL", spec)
        else:
            monkeypatch.delenv("GJ_TEST_ALLOC_FAIL", raising=False)
        return GaussJordan(block_size=64, ranks=3, device="gpu", dtype=dtype, comm="async").run(
            700, gen="random", seed=4)
    full, streamed = run(""), run("2:residual")
    assert full["status"] == 0 and streamed["status"] == 0 and streamed["residual_fp64"]
    assert abs(streamed["residual"] - full["residual"]) <= 0.05 * full["residual"]
