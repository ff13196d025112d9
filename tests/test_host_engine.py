"""The native engine on the host executor (CPU): protocol, pivoting, numerics vs the numpy oracle
and numpy.linalg.inv on the reference's acceptance grid."""
import numpy as np
import pytest

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd.models.gauss_jordan import SingularMatrixError
from mpi_jordan_crazy_acceleration_amd.utils import gauss_jordan_reference, generate_matrix


def _mat(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "rand":
        return rng.standard_normal((n, n))
    if kind == "perm":  # reversed-identity dominant: forces off-diagonal pivots (row swaps)
        return np.eye(n)[::-1] + 0.01 * rng.standard_normal((n, n))
    return generate_matrix(n, kind)


GRID = [(12, 3), (10, 3), (11, 4), (10, 12), (10, 1), (7, 7), (37, 5)]


@pytest.mark.parametrize("n,m", GRID)
@pytest.mark.parametrize("p", [1, 2, 3, 5])
@pytest.mark.parametrize("kind", ["rand", "perm", "absdiff"])
def test_inverse_grid(n, m, p, kind):
    A = _mat(kind, n, seed=n * 31 + m)
    inv = gj.inverse(A, block_size=m, device="cpu", ranks=p)
    ref = np.linalg.inv(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-10


@pytest.mark.parametrize("p", [1, 2, 3, 4])
def test_matches_reference_oracle_and_pivots(p):
    n, m = 48, 4
    A = _mat("perm", n, 3)
    ref_inv, ref_piv = gauss_jordan_reference(A, m, p)
    rep = gj.GaussJordan(block_size=m, ranks=p, device="cpu").run(n, input=A, keep_inverse=True)
    assert rep["status"] == 0
    assert np.abs(rep["inverse"] - ref_inv).max() < 1e-11
    # same pivot *content*: the engine reports physical rows, the oracle logical positions after swaps
    assert rep["stats"]["offdiag_pivots"] > 0


@pytest.mark.parametrize("p,expected_first", [(1, 0), (2, 1), (3, 2), (4, 3)])
def test_pivot_tie_rule(p, expected_first):
    # all column-0 candidate blocks equal 2I -> ties go to the highest rank, then the
    # lowest local row: p=1 -> row 0, p=2 -> 1, p=3 -> 2, p=4 -> 3.
    m, Nr = 2, 4
    n = m * Nr
    A = np.zeros((n, n))
    for i in range(Nr):
        A[i * m:(i + 1) * m, 0:m] = 2 * np.eye(m)
    A[:, m:] = np.random.default_rng(5).standard_normal((n, n - m))
    rep = gj.GaussJordan(block_size=m, ranks=p, device="cpu").run(n, input=A, keep_inverse=True)
    assert rep["status"] == 0
    assert rep["stats"]["pivots"][0] == expected_first
    _, ref_piv = gauss_jordan_reference(A, m, p)
    assert ref_piv[0] == expected_first
    assert np.abs(rep["inverse"] - np.linalg.inv(A)).max() < 1e-10


def test_singular_matrix_reported():
    with pytest.raises(SingularMatrixError):
        gj.inverse(np.zeros((2, 2)), block_size=1, device="cpu")
    A = _mat("rand", 20, 1)
    A[:, 3] = 0
    rep = gj.GaussJordan(block_size=4, ranks=2, device="cpu").run(20, input=A)
    assert rep["status"] == 1 and rep["status_name"] == "singular matrix"


def test_two_by_two_reference_case():
    inv = gj.inverse(np.array([[1.0, 2.0], [3.0, 4.0]]), block_size=1, device="cpu")
    assert np.allclose(inv, [[-2, 1], [1.5, -0.5]], atol=1e-14)


@pytest.mark.parametrize("n,m,p,golden", [(12, 3, 2, 4.550968e-14), (10, 3, 2, 3.053268e-14), (11, 4, 2, 1.192324e-13)])
def test_absdiff_golden_residual_band(n, m, p, golden):
    rep = gj.run(n, m, ranks=p, device="cpu", gen="absdiff")
    assert rep["status"] == 0
    assert rep["residual"] < 20 * golden


def test_absdiff_residual_no_worse_than_reference_n2048():
    # reference: n=2048, m=120, p=8 -> 1.85e-06
    rep = gj.run(2048, 120, ranks=4, device="cpu", gen="absdiff", host_threads=2)
    assert rep["status"] == 0 and rep["residual"] < 1.85e-6


def test_hilbert_and_fp32():
    rep = gj.run(8, 2, device="cpu", gen="hilbert")
    assert rep["status"] == 0 and rep["residual"] < 1e-4
    rep = gj.run(200, 32, ranks=2, device="cpu", gen="random", seed=3, dtype="fp32")
    assert rep["status"] == 0 and rep["residual"] < 0.5  # fp32: eps 6e-8 x the fp64 amplification (~1e7)


def test_sync_debug_is_bitwise_identical():
    A = _mat("rand", 90, 7)
    a = gj.GaussJordan(block_size=8, ranks=3, device="cpu").inverse(A)
    b = gj.GaussJordan(block_size=8, ranks=3, device="cpu", sync_debug=True).inverse(A)
    assert np.array_equal(a, b)


def test_chunking_does_not_change_result():
    A = _mat("rand", 160, 9)
    a = gj.GaussJordan(block_size=8, device="cpu", chunk_cols=8).inverse(A)
    b = gj.GaussJordan(block_size=8, device="cpu", chunk_cols=160).inverse(A)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("ranks", [1, 2])
def test_uneven_chunk_plan_does_not_change_result(monkeypatch, ranks):
    # GJ_CHUNK_PLAN: explicit, uneven column chunks (block counts; multiples of the depth)
    A = _mat("rand", 160, 9)
    a = gj.GaussJordan(block_size=8, ranks=ranks, device="cpu", depth=2).inverse(A)
    monkeypatch.setenv("GJ_CHUNK_PLAN", "6,10,4")
    b = gj.GaussJordan(block_size=8, ranks=ranks, device="cpu", depth=2).inverse(A)
    assert np.array_equal(a, b)
    monkeypatch.setenv("GJ_CHUNK_PLAN", "6,10,5")
    with pytest.raises(Exception, match="GJ_CHUNK_PLAN"):
        gj.GaussJordan(block_size=8, ranks=ranks, device="cpu", depth=2).inverse(A)


def test_solve_rhs():
    A = _mat("rand", 64, 11)
    x = np.arange(64.0)
    b = A @ x
    got = gj.solve(A, b, block_size=16, device="cpu")
    assert np.abs(got - x).max() < 1e-9


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("n,m,p", [(37, 5, 1), (37, 5, 3), (64, 8, 2), (10, 3, 4), (50, 7, 5), (12, 12, 2)])
@pytest.mark.parametrize("kind", ["rand", "perm"])
def test_depth_variants_match_numpy(depth, n, m, p, kind):
    A = _mat(kind, n, seed=n + m + p)
    inv = gj.GaussJordan(block_size=m, ranks=p, device="cpu", depth=depth, chunk_cols=2 * m).inverse(A)
    ref = np.linalg.inv(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-10


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_depth_absdiff_residual_matches_reference_band(depth):
    rep = gj.run(512, 64, ranks=2, device="cpu", gen="absdiff", depth=depth)
    assert rep["status"] == 0 and rep["residual"] < 5e-8


def test_depth_pivots_identical():
    A = _mat("perm", 64, 4)
    p1 = gj.GaussJordan(block_size=4, ranks=3, device="cpu", depth=1).run(64, input=A)["stats"]["pivots"]
    p3 = gj.GaussJordan(block_size=4, ranks=3, device="cpu", depth=3).run(64, input=A)["stats"]["pivots"]
    assert p1 == p3


def test_host_gemm_extras_match_torch():
    import torch
    from mpi_jordan_crazy_acceleration_amd import ops
    g = torch.Generator().manual_seed(3)
    A = torch.rand(90, 20, generator=g, dtype=torch.float64)
    B = torch.rand(20, 70, generator=g, dtype=torch.float64)
    C = torch.rand(90, 70, generator=g, dtype=torch.float64)
    Cin = C.clone()
    Cin[:, 5:25] = 0
    Cin[30:40] = 0
    ref = Cin + A @ B
    ops.gemm(A.t().contiguous(), B, C, op="acc", a_kmajor=True, zero_cols=(5, 25), zero_rows=[30], zero_row_height=10)
    assert (C - ref).abs().max().item() < 1e-12


def test_host_gemm_tneg_epilogue():
    """Host executor: the column update's fused multiplier write, tneg = -C^T after C += A B."""
    import torch
    from mpi_jordan_crazy_acceleration_amd import ops
    g = torch.Generator().manual_seed(4)
    A = torch.rand(90, 20, generator=g, dtype=torch.float64)
    B = torch.rand(20, 70, generator=g, dtype=torch.float64)
    C = torch.rand(90, 70, generator=g, dtype=torch.float64)
    ref = C + A @ B
    T = torch.full((70, 96), 3.0, dtype=torch.float64)
    ops.gemm(A.t().contiguous(), B, C, op="acc", a_kmajor=True, tneg=T[:, :90])
    assert (C - ref).abs().max().item() < 1e-12
    assert torch.equal(T[:, :90], -C.t())
    assert torch.equal(T[:, 90:], torch.full((70, 6), 3.0, dtype=torch.float64))
    T2 = torch.full((70, 90), 5.0, dtype=torch.float64)
    C2 = torch.rand(90, 70, generator=g, dtype=torch.float64)
    ops.gemm(A.t().contiguous(), B, C2, op="acc", a_kmajor=True, tneg=T2[:30])
    assert torch.equal(T2[:30], -C2.t()[:30]) and torch.equal(T2[30:], torch.full((40, 90), 5.0, dtype=torch.float64))


def test_python_solve_vector_native_path(native):
    import mpi_jordan_crazy_acceleration_amd as gj
    rng = np.random.default_rng(11)
    A = rng.standard_normal((70, 70))
    b = rng.standard_normal(70)
    x = gj.solve(A, b, block_size=16, device="cpu", ranks=3)
    assert np.abs(A @ x - b).max() < 1e-10
    X = gj.solve(A, np.stack([b, 2 * b], 1), block_size=16, device="cpu")
    assert np.allclose(X[:, 1], 2 * x, atol=1e-9)


def test_engine_profile_phases(native):
    rep = native.run_local(dict(n=150, m=16, ranks=2, device="cpu", gen="random", profile=True,
                                rhs="ones"))
    ph = rep["stats"]["phases"]
    assert ph["trailing_update"]["calls"] > 0 and ph["pivot_search"]["calls"] == 10
    assert rep["axb_residual"] < 1e-10


def test_loopback_detects_collective_mismatch(native):
    ok = native.loopback_mismatch_probe(0)
    assert ok == ["", ""]
    bad = native.loopback_mismatch_probe(1)
    assert all("collective mismatch" in m for m in bad), bad


def test_rows_device_io_on_host_executor(native):
    """upload_rows_device / download_rows_device (the zero-copy path used for CUDA tensors) on the
    host executor, where the "device" pointers are host arrays."""
    n, m = 90, 16
    A = _mat("rand", n, 5)
    eng = native.Engine(native.host_device(2), native.self_comm(), n, m, "fp64")
    src = np.zeros((n, n + 3))
    src[:, :n] = A
    eng.upload_rows_device(src.ctypes.data, n + 3)
    assert eng.solve()["status"] == 0
    out = np.full((n, n + 5), np.nan)
    eng.download_rows_device(out.ctypes.data, n + 5)
    assert np.abs(out[:, :n] - np.linalg.inv(A)).max() / np.abs(np.linalg.inv(A)).max() < 1e-10
    assert np.isnan(out[:, n:]).all()


def test_host_gemm_batch_matches_torch():
    import torch
    from mpi_jordan_crazy_acceleration_amd import ops
    g = torch.Generator().manual_seed(5)
    prods, refs = [], []
    for i, (M, N, K) in enumerate([(16, 16, 48), (16, 40, 32), (9, 7, 5)]):
        At = torch.rand(K, M, generator=g, dtype=torch.float64)
        B = torch.rand(K, N, generator=g, dtype=torch.float64)
        C = torch.rand(M, N, generator=g, dtype=torch.float64)
        op = "store" if i != 1 else "acc"
        refs.append(At.t() @ B + (C if op == "acc" else 0))
        prods.append((op, At, B, C))
    ops.gemm_batch(prods)
    for (_, _, _, C), r in zip(prods, refs):
        assert (C - r).abs().max().item() < 1e-12


def test_unknown_variant_names_fail_loudly(native):
    """A typo'd GEMM or block-inverse variant name is an error, never a silent default."""
    with pytest.raises(ValueError, match="unknown GEMM variant"):
        native.set_gemm_variant("dtva")
    with pytest.raises(ValueError, match="unknown block-inverse variant"):
        native.set_block_inverse_variant("pannel")
    native.set_gemm_variant("auto")
    native.set_block_inverse_variant("panel")


@pytest.mark.parametrize("first", [1, 2, 3])
@pytest.mark.parametrize("depth", [2, 4, 6])
@pytest.mark.parametrize("n,m,p", [(37, 5, 1), (37, 5, 3), (64, 8, 2), (50, 7, 5), (12, 12, 2)])
def test_shallow_first_panel_matches_numpy(monkeypatch, first, depth, n, m, p):
    # GJ_FIRST_DEPTH: panel 0 takes `first` steps (capped at the depth), every later one `depth`;
    # chunk boundaries move onto the shifted panel boundaries; GJ_VERIFY checks every hand-over
    monkeypatch.setenv("GJ_FIRST_DEPTH", str(first))
    monkeypatch.setenv("GJ_VERIFY", "1")
    A = _mat("perm", n, seed=n + m + p + first)
    g = gj.GaussJordan(block_size=m, ranks=p, device="cpu", depth=depth, chunk_cols=2 * m)
    inv = g.inverse(A)
    ref = np.linalg.inv(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-10


def test_shallow_first_panel_chunk_plan(monkeypatch):
    # explicit plans must end on the shifted panel boundaries (1 + 2k for first depth 1, depth 2)
    A = _mat("rand", 160, 9)
    ref = np.linalg.inv(A)
    monkeypatch.setenv("GJ_FIRST_DEPTH", "1")
    monkeypatch.setenv("GJ_CHUNK_PLAN", "7,10,3")
    inv = gj.GaussJordan(block_size=8, device="cpu", depth=2).inverse(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-10
    monkeypatch.setenv("GJ_CHUNK_PLAN", "6,10,4")
    with pytest.raises(Exception, match="GJ_CHUNK_PLAN"):
        gj.GaussJordan(block_size=8, device="cpu", depth=2).inverse(A)


@pytest.mark.parametrize("split", ["1", "2"])
@pytest.mark.parametrize("skip", ["0", "1"])
@pytest.mark.parametrize("ranks", [1, 3])
def test_main_split_launches_bit_identical(monkeypatch, split, skip, ranks):
    # GJ_MAIN_SPLIT: MAIN's chunk updates in two column halves (with and without the look-ahead
    # skip inside one launch): the same products per element, so the same bits
    A = _mat("rand", 1100, 13)
    monkeypatch.setenv("GJ_SKIP_COLS", skip)
    a = gj.GaussJordan(block_size=10, ranks=ranks, device="cpu", depth=4, chunk_cols=600).inverse(A)
    monkeypatch.setenv("GJ_MAIN_SPLIT", split)
    b = gj.GaussJordan(block_size=10, ranks=ranks, device="cpu", depth=4, chunk_cols=600).inverse(A)
    assert np.array_equal(a, b)
    assert np.abs(a @ A - np.eye(1100)).max() < 1e-8
