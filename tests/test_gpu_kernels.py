"""Per-kernel numerics on the MI355X: every hand-written HIP kernel vs a plain PyTorch/numpy fp64
reference of the same op (asymmetric operands, ragged edges)."""
import numpy as np
import pytest
import torch

import mpi_jordan_crazy_acceleration_amd as gj
from mpi_jordan_crazy_acceleration_amd import ops
from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix

pytestmark = pytest.mark.gpu


def _rand(shape, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1).to(dtype)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (256, 384, 128), (300, 200, 60), (37, 515, 17), (1000, 130, 256), (2100, 1600, 136)])
@pytest.mark.parametrize("kmajor", [True, False])
def test_gemm_acc_matches_torch(dtype, M, N, K, kmajor):
    A = _rand((M, K), dtype, 1)
    B = _rand((K, N), dtype, 2)
    C = _rand((M, N), dtype, 3)
    ref = C.double() + A.double() @ B.double()
    Ad = (A.t().contiguous() if kmajor else A).cuda()
    Cd = C.cuda()
    ops.gemm(Ad, B.cuda(), Cd, op="acc", a_kmajor=kmajor)
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    err = (Cd.cpu().double() - ref).abs().max().item()
    assert err < tol * K, err


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_gemm_store_identity_asymmetric(dtype):
    # A = I with an asymmetric B catches a transposed C/D lane map (guide §3)
    M = N = K = 128
    A = torch.eye(M, dtype=dtype)
    B = torch.arange(K * N, dtype=dtype).reshape(K, N) / 7.0
    C = torch.full((M, N), 5.0, dtype=dtype).cuda()
    ops.gemm(A.cuda(), B.cuda(), C, op="store", a_kmajor=True)
    assert torch.equal(C.cpu(), B)


def test_generate_matches_numpy():
    n, m = 300, 64
    Nr = (n + m - 1) // m
    X = torch.empty((Nr * m, Nr * m), dtype=torch.float64, device="cuda")
    ops.generate(X, n, m, 1, 0, "random", 11)
    ref = generate_matrix(n, "random", 11)
    Xc = X.cpu().numpy()
    assert np.array_equal(Xc[:n, :n], ref)
    assert np.array_equal(Xc[n:, n:], np.eye(Nr * m - n))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("M,K,latency,variant,N,tcols", [(300, 256, True, "auto", 128, 128),
                                                          (4096, 384, True, "auto", 128, 128),
                                                          (1000, 512, False, "auto", 128, 128),
                                                          (777, 128, False, "glds", 128, 128),
                                                          (2048, 256, False, "big", 128, 128),
                                                          (513, 128, True, "narrow", 128, 128),
                                                          (1000, 256, False, "glds", 512, 128),
                                                          (16384, 512, False, "auto", 512, 128),
                                                          (1030, 256, False, "narrow", 384, 100)])
def test_gemm_tneg_epilogue(native, dtype, M, K, latency, variant, N, tcols):
    """Column / look-ahead update with the fused multiplier write: C += A B and tneg = -C^T of the
    first tcols columns (bit-identical to C), on every tile family incl. the LDS-DMA kernel."""
    native.set_gemm_variant(variant)
    try:
        At = _rand((K, M), dtype, 21).cuda()
        B = _rand((K, N), dtype, 22).cuda()
        C = _rand((M, N), dtype, 23)
        ref = C.double() + At.cpu().double().t() @ B.cpu().double()
        Cd = C.cuda()
        T = torch.full((N, M + 8), 7.0, dtype=dtype, device="cuda")
        ops.gemm(At, B, Cd, op="acc", a_kmajor=True, tneg=T[:tcols, :M],
                 latency=latency)
        tol = (1e-12 if dtype == torch.float64 else 2e-5) * K
        assert (Cd.cpu().double() - ref).abs().max().item() < tol
        assert torch.equal(T[:tcols, :M].cpu(), -Cd.cpu().t()[:tcols])
        assert torch.equal(T[:tcols, M:].cpu(), torch.full((tcols, 8), 7.0, dtype=dtype))
        assert torch.equal(T[tcols:].cpu(), torch.full((N - tcols, M + 8), 7.0, dtype=dtype))
    finally:
        native.set_gemm_variant("auto")


def test_extract_neg_t():
    X = _rand((300, 512), torch.float64, 5).cuda()
    Lt = ops.extract_neg_t(X, 128, 96)
    assert torch.equal(Lt.cpu(), -X.cpu()[:, 128:224].t())


@pytest.fixture(params=["panel", "sweep", "co", "generic"])
def bi_variant(request, native):
    native.set_block_inverse_variant(request.param)
    yield request.param
    native.set_block_inverse_variant("panel")


@pytest.mark.parametrize("m", [16, 37, 60, 64, 100, 128, 200, 256, 300, 512, 700, 1000])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_block_inverse(m, dtype, bi_variant):
    nblk = 6
    rows = nblk * m
    rng = np.random.default_rng(m)
    W = rng.standard_normal((nblk, m, m)) + 0.0
    W[2] = 0.0  # singular candidate
    W[3] = np.eye(m) * 2.0  # exact inverse 0.5 I
    W[5][:, m // 2] = 0.0  # exactly singular part-way through the sweep
    X = np.zeros((rows, m))
    for b in range(nblk):
        X[b * m:(b + 1) * m] = W[b]
    Lt = torch.from_numpy(-X.T.copy()).to(dtype).cuda()
    n = rows
    inv_t, scores, valid = ops.block_inverse(Lt, n, m, 1, 0, thresh=1e-12)
    valid = valid.cpu().numpy()
    assert list(valid) == [1, 1, 0, 1, 1, 0]
    tol = 1e-8 if dtype == torch.float64 else 2e-2
    for b in [0, 1, 3, 4]:
        ref = np.linalg.inv(W[b].astype(np.float32 if dtype == torch.float32 else np.float64).astype(np.float64))
        got = inv_t[b].cpu().double().numpy().T
        rel = np.abs(got - ref).max() / np.abs(ref).max()
        assert rel < tol, (b, rel)
        assert abs(scores[b].item() - np.abs(ref).sum(1).max()) / np.abs(ref).sum(1).max() < tol
    assert abs(scores[3].item() - 0.5) < 1e-6


@pytest.mark.parametrize("m,dtype", [(300, torch.float64), (1000, torch.float64), (2500, torch.float64),
                                     (700, torch.float32), (4608, torch.float64)])
def test_block_inverse_huge_gpu_wide(native, m, dtype):
    """The GPU-wide candidate inverse (panel factor on one workgroup + MFMA GEMM updates, the default
    above m = 4096, forced with variant "huge" below): against numpy, with a singular block in the
    batch, and against the panel-blocked kernel where that one applies (same pivot rule: inverses
    and scores agree to rounding)."""
    nblk = 3 if m <= 2500 else 2
    rng = np.random.default_rng(m + 11)
    W = rng.standard_normal((nblk, m, m))
    if dtype == torch.float32:
        W += np.sqrt(m) * np.eye(m)
    W[1] = 0.0
    X = W.reshape(nblk * m, m)
    Lt = torch.from_numpy(-X.T.copy()).to(dtype).cuda()
    native.set_block_inverse_variant("huge")
    try:
        inv_h, scores_h, valid_h = ops.block_inverse(Lt, nblk * m, m, 1, 0, thresh=1e-12)
    finally:
        native.set_block_inverse_variant("panel")
    assert valid_h.cpu().tolist()[:2] == [1, 0]
    tol = 1e-9 if dtype == torch.float64 else 1e-4
    for b in [x for x in range(nblk) if x != 1]:
        ref = np.linalg.inv(W[b].astype(np.float32 if dtype == torch.float32 else np.float64).astype(np.float64))
        got = inv_h[b].cpu().double().numpy().T
        assert np.abs(got - ref).max() / np.abs(ref).max() < tol
        assert abs(scores_h[b].item() / np.abs(ref).sum(1).max() - 1) < tol * 10
    if m <= 4096:  # the panel-blocked kernel (or the matrix-core one) on the same batch
        inv_p, scores_p, valid_p = ops.block_inverse(Lt, nblk * m, m, 1, 0, thresh=1e-12)
        assert valid_p.cpu().tolist() == valid_h.cpu().tolist()
        for b in (0, 2):
            a, c = inv_h[b].cpu().double(), inv_p[b].cpu().double()
            assert ((a - c).abs().max() / c.abs().max()).item() < tol
            assert abs(scores_h[b].item() / scores_p[b].item() - 1) < tol * 10


@pytest.mark.parametrize("n,m", [(5000, 5000), (9000, 4500)])
def test_engine_block_size_above_4096(n, m):
    """m > 4096 in the solver (the reference inverts any m, main.cpp:746-820): one or two block rows,
    every candidate inverse on the GPU-wide path; the inverse against numpy."""
    A = generate_matrix(n, "random", 23)
    inv = gj.GaussJordan(block_size=m, ranks=1, device="gpu").inverse(A)
    ref = np.linalg.inv(A)
    assert np.abs(inv - ref).max() / np.abs(ref).max() < 1e-8 * max(1.0, m / 256)


@pytest.mark.parametrize("m,dtype", [(2500, torch.float64), (4096, torch.float32)])
def test_block_inverse_large_m_panel_blocked(native, m, dtype):
    """2048 < m <= 4096: the panel-blocked kernel with 12 / 16 rows per thread and 2-column panels
    (was the per-step global sweep), against numpy and against that sweep (the same pivot rule:
    the inverses and scores agree to rounding)."""
    nblk = 3
    rng = np.random.default_rng(m)
    W = rng.standard_normal((nblk, m, m))
    if dtype == torch.float32:
        W += np.sqrt(m) * np.eye(m)  # an fp32 inverse of a random block this size is meaningless
    W[1] = 0.0
    X = W.reshape(nblk * m, m)
    Lt = torch.from_numpy(-X.T.copy()).to(dtype).cuda()
    native.set_block_inverse_variant("blocked")  # (the default takes the GPU-wide form for few candidates)
    try:
        inv_t, scores, valid = ops.block_inverse(Lt, nblk * m, m, 1, 0, thresh=1e-12)
        native.set_block_inverse_variant("generic")
        inv_g, scores_g, valid_g = ops.block_inverse(Lt, nblk * m, m, 1, 0, thresh=1e-12)
    finally:
        native.set_block_inverse_variant("panel")
    assert valid.cpu().tolist() == [1, 0, 1] and valid_g.cpu().tolist() == [1, 0, 1]
    tol = 1e-9 if dtype == torch.float64 else 1e-4
    for b in (0, 2):
        ref = np.linalg.inv(W[b].astype(np.float32 if dtype == torch.float32 else np.float64).astype(np.float64))
        got = inv_t[b].cpu().double().numpy().T
        assert np.abs(got - ref).max() / np.abs(ref).max() < tol
        gen = inv_g[b].cpu().double().numpy().T
        assert np.abs(got - gen).max() / np.abs(gen).max() < tol
        assert abs(scores[b].item() - scores_g[b].item()) <= tol * scores_g[b].item()


@pytest.mark.parametrize("m,blocks,latency", [(64, [0, 2, 3, 7], True), (128, [1, 4], False), (128, [0], True),
                                              (64, list(range(8)), False), (128, [0, 3, 5, 6, 7], True)])
@pytest.mark.parametrize("c_in", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("lat_glds", [False, True])
def test_gemm_row_blocks_and_c_in(m, blocks, latency, c_in, dtype, lat_glds, native):
    """GemmExtra::rsel (the split pivot chain's row-selected column updates) and GemmExtra::c_in (the
    owners' normalisation input without a copy): only the selected row blocks of C and -C^T change,
    with C_in + A B; the others keep their bytes.  Same k order as the full product: bit-identical
    rows.  128-row blocks take the LDS-DMA kernel (latency launches too with set_lat_glds)."""
    native.set_lat_glds(lat_glds)
    try:
        _row_blocks_case(m, blocks, latency, c_in, dtype)
    finally:
        native.set_lat_glds(False)


def _row_blocks_case(m, blocks, latency, c_in, dtype):
    M, N, K = 8 * m, 192, 3 * m
    A = _rand((M, K), torch.float64, 41).to(dtype).cuda()
    B = _rand((K, N), torch.float64, 42).to(dtype).cuda()
    C = _rand((M, N), torch.float64, 43).to(dtype).cuda()
    Ci = _rand((M, N), torch.float64, 44).to(dtype).cuda() if c_in else None
    T = torch.full((m, M), 5.0, dtype=dtype, device="cuda")
    full = (Ci if c_in else C).clone()
    Tf = T.clone()
    ops.gemm(A.t().contiguous(), B, full, op="acc", a_kmajor=True, tneg=Tf, latency=latency)
    got = C.clone()
    ops.gemm(A.t().contiguous(), B, got, op="acc", a_kmajor=True, tneg=T, latency=latency, c_in=Ci,
             row_blocks=blocks, row_block_m=m)
    sel = torch.zeros(M, dtype=torch.bool)
    for b in blocks:
        sel[b * m:(b + 1) * m] = True
    sel = sel.cuda()
    assert torch.equal(got[sel], full[sel])
    assert torch.equal(got[~sel], C[~sel])
    assert torch.equal(T[:, sel], Tf[:, sel]) and bool((T[:, ~sel] == 5.0).all())


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("m", [32, 33, 60, 128, 300])
def test_permute_blocks(m, dtype):
    # the 16-byte kernel where a column block's bytes and the leading dimensions are multiples of 16
    # (every m here but 33), the scalar one otherwise
    nblk, Nr = 3, 5
    X = _rand((nblk * m, Nr * m), dtype, 9).cuda()
    dst = torch.tensor([2, 0, 1], dtype=torch.int32, device="cuda")
    colsrc = torch.tensor([4, 3, 0, 1, 2], dtype=torch.int32, device="cuda")
    out = ops.permute_blocks(X, m, dst, colsrc).cpu()
    Xc = X.cpu()
    for b in range(nblk):
        for c in range(Nr):
            d = int(dst[b])
            u = int(colsrc[c])
            assert torch.equal(out[d * m:(d + 1) * m, c * m:(c + 1) * m], Xc[b * m:(b + 1) * m, u * m:(u + 1) * m])


def test_row_abs_max_and_residual():
    n, m = 250, 64
    A = generate_matrix(n, "random", 3)
    Nr = (n + m - 1) // m
    npad = Nr * m
    Ap = np.eye(npad)
    Ap[:n, :n] = A
    inv = np.eye(npad)
    inv[:n, :n] = np.linalg.inv(A)
    Ad = torch.from_numpy(Ap).cuda()
    assert abs(ops.row_abs_max(Ad, n, m) - np.abs(A).sum(1).max()) < 1e-9
    r = ops.residual(Ad, torch.from_numpy(inv).cuda(), n, m)
    ref = np.abs(A @ np.linalg.inv(A) - np.eye(n)).sum(1).max()
    assert r < 1e-10 and abs(r - ref) < 1e-11


GEMM_VARIANTS = ["big", "narrow", "squarepf", "bigpf", "auto", "glds"]


@pytest.mark.parametrize("variant", GEMM_VARIANTS)
@pytest.mark.parametrize("M,N,K", [(256, 384, 128), (300, 200, 60), (1000, 130, 256), (2100, 1600, 136),
                                   (700, 1100, 512), (1536, 1024, 520)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_gemm_variants_elimination_extras(native, variant, M, N, K, dtype):
    """All kernel variants: C += A B where C enters as 0 in a column range and in two row blocks."""
    native.set_gemm_variant(variant)
    try:
        A = _rand((M, K), torch.float64, 11)
        B = _rand((K, N), torch.float64, 12)
        C = _rand((M, N), torch.float64, 13)
        z0, z1, zr, zh = 17, 17 + K // 2, [70, 190], 45
        Cin = C.clone()
        Cin[:, z0:z1] = 0
        for r in zr:
            Cin[r:r + zh] = 0
        ref = Cin + A @ B
        tol = (1e-12 if dtype == torch.float64 else 2e-5) * K
        Cd = C.to(dtype).cuda()
        ops.gemm(A.t().contiguous().to(dtype).cuda(), B.to(dtype).cuda(), Cd, op="acc", a_kmajor=True,
                 zero_cols=(z0, z1), zero_rows=zr, zero_row_height=zh)
        assert (Cd.cpu().double() - ref).abs().max().item() < tol
        Cs = torch.zeros(M, N, dtype=dtype).cuda()
        ops.gemm(A.t().contiguous().to(dtype).cuda(), B.to(dtype).cuda(), Cs, op="store", a_kmajor=True)
        assert (Cs.cpu().double() - A @ B).abs().max().item() < tol
    finally:
        native.set_gemm_variant("auto")


@pytest.mark.parametrize("M,N,K", [(2948, 2900, 520), (2950, 2900, 520), (2948, 2902, 1000)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("variant", ["auto", "glds"])
def test_gemm_deep_auto_dispatch(native, M, N, K, dtype, variant):
    """Deep updates with enough tiles take the LDS-DMA kernels under "auto" (fp32: the 32x32x2 one
    when M, N are multiples of 4, else the register-staged tile) and under an explicit "glds":
    ragged edges, zero extras."""
    native.set_gemm_variant(variant)
    A = _rand((M, K), torch.float64, 21)
    B = _rand((K, N), torch.float64, 22)
    C = _rand((M, N), torch.float64, 23)
    z0, z1, zr, zh = 128, 256, [0, 1000], 128
    Cin = C.clone()
    Cin[:, z0:z1] = 0
    for r in zr:
        Cin[r:r + zh] = 0
    ref = Cin + A @ B
    tol = (1e-12 if dtype == torch.float64 else 2e-5) * K
    Cd = C.to(dtype).cuda()
    try:
        ops.gemm(A.t().contiguous().to(dtype).cuda(), B.to(dtype).cuda(), Cd, op="acc", a_kmajor=True,
                 zero_cols=(z0, z1), zero_rows=zr, zero_row_height=zh)
    finally:
        native.set_gemm_variant("auto")
    assert (Cd.cpu().double() - ref).abs().max().item() < tol


@pytest.mark.parametrize("M,N,K", [(2948, 2900, 520), (2050, 1030, 516), (1538, 2050, 1003), (4096, 2048, 256),
                                   (2048, 1024, 8), (1026, 514, 20), (2948, 2902, 16)])
@pytest.mark.parametrize("build", [23, 33, 25])
def test_glds_peeled_loop_matches_reference(native, M, N, K, build):
    """The fp64 LDS-DMA trailing update with the peeled, stage-unrolled main loop (set_glds_peel):
    K multiple of the 8-deep slice or not (the partial last slice takes the masked issue), too
    short for a steady-state trip, every build (2 / 3 stages, 4 and 5 per CU); ragged M / N edges,
    zero extras.  Bit-identical to the general loop of the same build."""
    A = _rand((M, K), torch.float64, 31)
    B = _rand((K, N), torch.float64, 32)
    C = _rand((M, N), torch.float64, 33)
    z0, z1, zr, zh = 128, 256, [0, 1000], 128
    Cin = C.clone()
    Cin[:, z0:z1] = 0
    for r in zr:
        Cin[r:r + zh] = 0
    ref = Cin + A @ B
    outs = []
    native.set_glds_build(build)
    try:
        for peel in (0, 1):
            native.set_glds_peel(peel)
            Cd = C.cuda()
            ops.gemm(A.t().contiguous().cuda(), B.cuda(), Cd, op="acc", a_kmajor=True, zero_cols=(z0, z1),
                     zero_rows=zr, zero_row_height=zh, dense=(build == 25))
            outs.append(Cd.cpu())
    finally:
        native.set_glds_peel(1)
        native.set_glds_build(0)
    assert (outs[1].double() - ref).abs().max().item() < 1e-12 * K
    # same k order, same MFMAs: the peeled loop is bit-identical to the general one
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K", [(2948, 2900, 520), (2050, 1030, 516), (1538, 2050, 1003), (4096, 2048, 512),
                                   (2048, 1024, 8), (1026, 514, 20), (2948, 2902, 16), (640, 200, 512)])
@pytest.mark.parametrize("build", [33, 23, 32])
def test_glds_tile128_matches_reference(native, M, N, K, build):
    """The 128 x 128 LDS-DMA tile (set_glds_tile(128): 2 x 2 waves of 64 x 64, one B DMA piece per
    k row) against the fp64 reference, with zero columns / rows, ragged edges, K not a multiple of
    the slice; bit-identical to the 128 x 64 tile (same MFMAs in the same k order per element)."""
    A = _rand((M, K), torch.float64, 41)
    B = _rand((K, N), torch.float64, 42)
    C = _rand((M, N), torch.float64, 43)
    z0, z1, zr, zh = 128, 256, [0, 384], 128
    Cin = C.clone()
    Cin[:, z0:z1] = 0
    for r in zr:
        Cin[r:r + zh] = 0
    ref = Cin + A @ B
    outs = []
    try:
        for tile in (64, 128):
            native.set_glds_tile(tile)
            native.set_glds_build(build if tile == 128 else 33)
            Cd = C.cuda()
            ops.gemm(A.t().contiguous().cuda(), B.cuda(), Cd, op="acc", a_kmajor=True, zero_cols=(z0, z1),
                     zero_rows=zr, zero_row_height=zh)
            outs.append(Cd.cpu())
    finally:
        native.set_glds_tile(0)  # per launch (the default)
        native.set_glds_build(0)
    assert (outs[1].double() - ref).abs().max().item() < 1e-12 * K
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 512), (2052, 1028, 520), (1028, 2060, 100), (640, 256, 512),
                                   (1024, 264, 16)])
def test_glds32_tile256_matches_reference(native, M, N, K):
    """The fp32 LDS-DMA kernel's 128 x 256 tile (taken where the wide fp64 tile is named,
    set_glds_tile(128): 2 x 2 waves of 64 x 128, one B DMA piece per k row) against an fp64
    reference and bit-identical to the 128 x 128 fp32 tile; zero columns / rows, ragged edges."""
    A = _rand((M, K), torch.float32, 51)
    B = _rand((K, N), torch.float32, 52)
    C = _rand((M, N), torch.float32, 53)
    z0, z1, zr, zh = 128, 256, [0, 512], 128
    Cin = C.double().clone()
    Cin[:, z0:z1] = 0
    for r in zr:
        Cin[r:r + zh] = 0
    ref = Cin + A.double() @ B.double()
    outs = []
    try:
        for tile in (64, 128):
            native.set_glds_tile(tile)
            Cd = C.cuda()
            ops.gemm(A.t().contiguous().cuda(), B.cuda(), Cd, op="acc", a_kmajor=True, zero_cols=(z0, z1),
                     zero_rows=zr, zero_row_height=zh)
            outs.append(Cd.cpu())
    finally:
        native.set_glds_tile(0)
    assert ((outs[1].double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    assert torch.equal(outs[0], outs[1])


def test_engine_tile128_bit_identical(native):
    """The whole solve with the 128 x 128 trailing-update tile: the same inverse bits as 128 x 64."""
    n, m = 4096, 128
    outs = []
    try:
        for tile in (64, 128):
            native.set_glds_tile(tile)
            eng = native.Engine(native.hip_device(0), native.self_comm(), n, m, "fp64", 0, 1e-15, False, 4)
            eng.generate("random", 3)
            assert eng.solve()["status"] == 0
            outs.append(eng.download_local_rows())
    finally:
        native.set_glds_tile(0)  # per launch (the default)
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("count", [1, 3, 4, 6])
def test_gemm_batch_mixed_store_acc(dtype, count):
    """Batched small products (one launch per 4): store and acc mixed, ragged shapes, views with
    leading dimensions of a shared buffer (the panel-piece layout)."""
    shapes = [(128, 128, 384), (128, 384, 256), (100, 70, 33), (128, 128, 128), (64, 200, 520), (1, 3, 5)]
    big = _rand((130, 900), dtype, 40).cuda()  # every C is a column window of this buffer
    ref = big.cpu().double().clone()
    prods, col = [], 0
    for i in range(count):
        M, N, K = shapes[i]
        At = _rand((K, M), dtype, 50 + i).cuda()
        B = _rand((K, 2 * N), dtype, 60 + i).cuda()[:, :N]
        op = "store" if i % 2 == 0 else "acc"
        C = big[:M, col:col + N]
        prod = At.cpu().double().t() @ B.cpu().double()
        ref[:M, col:col + N] = prod if op == "store" else ref[:M, col:col + N] + prod
        prods.append((op, At, B, C))
        col += N
        col = col % 600
    ops.gemm_batch(prods)
    tol = (1e-12 if dtype == torch.float64 else 2e-5) * 520
    assert (big.cpu().double() - ref).abs().max().item() < tol


def _reference_pivots(W):
    """Original row of the pivot of every column under the reference's scan (main.cpp:746-820):
    physical row swaps, the first maximum |value| among positions k..m-1 wins."""
    a = W.astype(np.float64).copy()
    m = a.shape[0]
    order = list(range(m))
    piv = []
    for k in range(m):
        r = k + int(np.argmax(np.abs(a[k:, k])))  # argmax: first maximum
        piv.append(order[r])
        a[[k, r]] = a[[r, k]]
        order[k], order[r] = order[r], order[k]
        a[k] = a[k] / a[k, k]
        for i in range(m):
            if i != k:
                a[i] = a[i] - a[i, k] * a[k]
    return piv


@pytest.mark.parametrize("m,dtype,variant", [
    (40, torch.float64, "panel"), (128, torch.float64, "panel"), (200, torch.float64, "panel"),
    (256, torch.float64, "panel"), (40, torch.float32, "panel"), (128, torch.float32, "panel"),
    (300, torch.float64, "panel"), (512, torch.float64, "panel"), (700, torch.float32, "panel"),
    (1000, torch.float64, "panel"),
    # the register sweep kernel: default for m <= 16 and fp32 128 < m <= 256, variant "sweep" else
    (16, torch.float64, "panel"), (200, torch.float32, "panel"), (128, torch.float64, "sweep"),
    (60, torch.float32, "sweep"),
    # the GPU-wide panel / GEMM form (m > 4096 by default; forced here)
    (300, torch.float64, "huge"), (700, torch.float32, "huge")])
def test_block_inverse_pivot_rule(native, m, dtype, variant):
    """exact magnitudes (ties resolved in the low word of the fp64 key) and, on
    equal magnitudes, the row at the lowest CURRENT position under the reference's swaps — in
    every candidate-inverse kernel."""
    native.set_block_inverse_variant(variant)
    rng = np.random.default_rng(7 + m)
    eps = 2.0 ** -51 if dtype == torch.float64 else 2.0 ** -22
    Ws = []
    # A: column 0 selects row 5 (rows 0 and 5 swap), column 1 then ties rows 0 and 3 at 2.0: the
    # reference takes position 3 (row 3); "lowest original row" would take row 0
    A = rng.uniform(-1, 1, (m, m))
    A[:, 0] = 0.0
    A[5, 0] = 4.0
    A[0, 1] = A[3, 1] = 2.0
    Ws.append(A)
    # B: near-equal magnitudes in column 0: row 7 is larger by one unit in the last place of the
    # row-2 value; row 1 has exactly row 7's magnitude (negative) and a lower position -> row 1
    B = rng.uniform(-1, 1, (m, m))
    B[2, 0] = 3.0
    B[7, 0] = 3.0 * (1 + eps)
    B[1, 0] = -3.0 * (1 + eps)
    Ws.append(B)
    nblk = len(Ws)
    X = np.concatenate(Ws, axis=0)
    Lt = torch.from_numpy(-X.T.copy()).to(dtype).cuda()
    probe = torch.full((nblk * m,), -1, dtype=torch.int32, device="cuda")
    native.set_block_inverse_probe(probe.data_ptr())
    try:
        inv_t, scores, valid = ops.block_inverse(Lt, nblk * m, m, 1, 0, thresh=1e-12)
        torch.cuda.synchronize()
    finally:
        native.set_block_inverse_probe(0)
        native.set_block_inverse_variant("panel")
    assert valid.cpu().tolist() == [1] * nblk
    got = probe.cpu().numpy().reshape(nblk, m)
    assert got[0][0] == 5 and got[0][1] == 3
    assert got[1][0] == 1
    for b, W in enumerate(Ws):
        ref = _reference_pivots(W.astype(np.float32).astype(np.float64) if dtype == torch.float32 else W)
        assert got[b].tolist()[:2] == ref[:2]
        # later columns: computed values (different operation order) may differ in the last bits,
        # so only the rule-determined prefix is pinned; the bulk must still agree
        assert np.mean(np.array(got[b]) == np.array(ref)) > 0.9


def _better(a, b, p):
    """pivot_better (gj/pivot.hpp; the reference's non-commutative MPI op, main.cpp:729-744)."""
    if not a["valid"]:
        return False
    if not b["valid"]:
        return True
    if a["score"] != b["score"]:
        return a["score"] < b["score"]
    ra, rb = a["logical"] % p, b["logical"] % p
    if ra != rb:
        return ra > rb
    return a["logical"] // p < b["logical"] // p


def _rec(buf):
    raw = buf.cpu().numpy().tobytes()
    score = np.frombuffer(raw[:8], dtype=np.float64)[0]
    logical, phys, valid, _ = np.frombuffer(raw[8:24], dtype=np.int32)
    return {"score": float(score), "logical": int(logical), "phys": int(phys), "valid": int(valid)}


@pytest.mark.parametrize("p,k", [(1, 0), (3, 1), (4, 3)])
def test_pivot_local_many_candidates(native, p, k):
    """nblk > 64 (every lane scans several candidates), used / invalid entries, exact
    score ties decided by the logical position — against the host rule."""
    m, nblk = 4, 200
    Nr = nblk * p
    rng = np.random.default_rng(11 + p)
    scores = rng.integers(1, 6, nblk).astype(np.float64)  # many exact ties
    valid = (rng.random(nblk) > 0.2).astype(np.int32)
    used = (rng.random(Nr) > 0.7).astype(np.int32)
    pos = rng.permutation(Nr).astype(np.int32)  # logical positions after earlier swaps
    dev = torch.device("cuda")
    t_s, t_v = torch.from_numpy(scores).to(dev), torch.from_numpy(valid).to(dev)
    t_u, t_p = torch.from_numpy(used).to(dev), torch.from_numpy(pos).to(dev)
    rec = torch.zeros(32, dtype=torch.uint8, device=dev)
    d = ops.device_for(t_s)
    d.pivot_local(t_s.data_ptr(), t_v.data_ptr(), t_u.data_ptr(), t_p.data_ptr(), Nr * m, m, p, k, rec.data_ptr())
    best = {"valid": 0, "score": 0.0, "logical": -1, "phys": -1}
    for b in range(nblk):
        g = b * p + k
        if used[g] or not valid[b]:
            continue
        c = {"valid": 1, "score": scores[b], "logical": int(pos[g]), "phys": g}
        if _better(c, best, p):
            best = c
    assert _rec(rec) == best


@pytest.mark.parametrize("p", [2, 8, 64, 130])
def test_pivot_global_records_and_host_mirror(native, p):
    """pivot_global (misc.hip): lane q reduces record q (p > 64: several per lane), exact score ties
    decided by the logical position, invalid records skipped; the winner's book-keeping and the
    pinned host mirror (relaxed system-scope stores, pivot_select.hpp) against the host rule."""
    rng = np.random.default_rng(40 + p)
    nr = 4 * p + 3  # block rows known to the book-keeping arrays
    t = 2
    logical = rng.permutation(np.arange(t, nr))[:p].astype(np.int32)  # distinct, not yet pivots
    raw = np.zeros((p, 32), dtype=np.uint8)
    recs = []
    for q in range(p):
        r = {"score": float(rng.integers(1, 4)), "logical": int(logical[q]), "phys": int(logical[q]),
             "valid": int(rng.random() > 0.25)}
        recs.append(r)
        raw[q, :8] = np.frombuffer(np.float64(r["score"]).tobytes(), dtype=np.uint8)
        raw[q, 8:24] = np.frombuffer(np.array([r["logical"], r["phys"], r["valid"], 0], dtype=np.int32).tobytes(),
                                     dtype=np.uint8)
    best = {"valid": 0, "score": 0.0, "logical": -1, "phys": -1}
    for r in recs:
        if _better(r, best, p):
            best = r
    dev = torch.device("cuda")
    t_r = torch.from_numpy(raw.reshape(-1)).to(dev)
    h_pos, h_phys = list(range(nr)), list(range(nr))
    pos = torch.tensor(h_pos, dtype=torch.int32, device=dev)
    phys_at = torch.tensor(h_phys, dtype=torch.int32, device=dev)
    used = torch.zeros(nr, dtype=torch.int32, device=dev)
    seq = torch.zeros(nr, dtype=torch.int32, device=dev)
    out = torch.zeros(32, dtype=torch.uint8, device=dev)
    d = ops.device_for(t_r)
    step, found, phys, owner, lg, score = d.pivot_global(t_r.data_ptr(), p, t, pos.data_ptr(), phys_at.data_ptr(),
                                                         used.data_ptr(), seq.data_ptr(), out.data_ptr())
    assert step == t
    if not best["valid"]:
        assert (found, phys, owner, lg) == (0, -1, -1, -1) and seq.cpu()[t] == -1
        return
    assert (found, phys, owner, lg, score) == (1, best["phys"], best["phys"] % p, best["logical"], best["score"])
    o = out.cpu().numpy().tobytes()
    assert tuple(np.frombuffer(o[:16], dtype=np.int32)) == (1, phys, owner, lg)
    assert np.frombuffer(o[16:24], dtype=np.float64)[0] == score and np.frombuffer(o[24:28], dtype=np.int32)[0] == t
    s = best["phys"]  # pivot_commit (gj/pivot.hpp)
    q, ls = h_phys[t], h_pos[s]
    h_pos[q] = ls
    h_phys[ls] = q
    h_pos[s] = t
    h_phys[t] = s
    assert pos.cpu().tolist() == h_pos and phys_at.cpu().tolist() == h_phys
    assert used.cpu().tolist()[s] == 1 and seq.cpu().tolist()[t] == s


def test_pivot_select_single_bookkeeping(native):
    m, nblk = 2, 150
    rng = np.random.default_rng(5)
    scores = rng.integers(1, 4, nblk).astype(np.float64)
    valid = np.ones(nblk, dtype=np.int32)
    valid[::7] = 0
    dev = torch.device("cuda")
    t_s, t_v = torch.from_numpy(scores).to(dev), torch.from_numpy(valid).to(dev)
    pos = torch.arange(nblk, dtype=torch.int32, device=dev)
    phys_at = torch.arange(nblk, dtype=torch.int32, device=dev)
    used = torch.zeros(nblk, dtype=torch.int32, device=dev)
    seq = torch.zeros(nblk, dtype=torch.int32, device=dev)
    rec = torch.zeros(32, dtype=torch.uint8, device=dev)
    out = torch.zeros(32, dtype=torch.uint8, device=dev)
    h_pos, h_phys, h_used, h_seq = list(range(nblk)), list(range(nblk)), [0] * nblk, [0] * nblk
    d = ops.device_for(t_s)
    for t in range(40):
        d.pivot_select_single(t_s.data_ptr(), t_v.data_ptr(), nblk * m, m, t, pos.data_ptr(), phys_at.data_ptr(),
                              used.data_ptr(), seq.data_ptr(), rec.data_ptr(), out.data_ptr())
        best = {"valid": 0, "score": 0.0, "logical": -1, "phys": -1}
        for b in range(nblk):
            if h_used[b] or not valid[b]:
                continue
            c = {"valid": 1, "score": scores[b], "logical": h_pos[b], "phys": b}
            if _better(c, best, 1):
                best = c
        assert _rec(rec) == best
        s = best["phys"]  # pivot_commit (gj/pivot.hpp)
        q, ls = h_phys[t], h_pos[s]
        h_pos[q] = ls
        h_phys[ls] = q
        h_pos[s] = t
        h_phys[t] = s
        h_used[s] = 1
        h_seq[t] = s
    assert pos.cpu().tolist() == h_pos and phys_at.cpu().tolist() == h_phys
    assert used.cpu().tolist() == h_used and seq.cpu().tolist()[:40] == h_seq[:40]


@pytest.mark.parametrize("variant,m,dtype", [("panel", 60, torch.float64), ("panel", 128, torch.float64),
                                             ("panel", 100, torch.float32), ("co", 128, torch.float64),
                                             ("panel", 256, torch.float64), ("panel", 300, torch.float64),
                                             ("panel", 1100, torch.float64), ("panel", 1700, torch.float32),
                                             ("sweep", 64, torch.float64), ("generic", 300, torch.float64),
                                             ("huge", 600, torch.float64)])
@pytest.mark.parametrize("p,k", [(1, 0), (3, 2)])
def test_block_inverse_live_grid_matches_full_grid(native, variant, m, dtype, p, k):
    """nlive >= 0 (the engine's launch): one workgroup per UNUSED candidate, the workgroup's block
    found from the used flags (live_block).  Every live block's inverse, score and validity must be
    bit-identical to the one-workgroup-per-block launch; used blocks are not touched."""
    rng = np.random.default_rng(m + p)
    nblk = 37 if m <= 300 else 9
    Nr = nblk * p
    Lt = torch.from_numpy(rng.uniform(-1, 1, (m, nblk * m))).to(dtype).cuda()
    used = torch.from_numpy((rng.random(Nr) < 0.5).astype(np.int32)).cuda()
    mine = used.cpu().numpy()[k::p][:nblk]
    live = np.flatnonzero(mine == 0)
    native.set_block_inverse_variant(variant)
    try:
        full = ops.block_inverse(Lt, Nr * m, m, p, k, used=used, thresh=1e-12)
        sentinel = [t.clone().fill_(7) for t in full]
        inv_t, scores, valid = [t.clone() for t in sentinel]
        device = ops.device_for(Lt)
        device.block_inverse(ops._DT[dtype], Lt.data_ptr(), Lt.stride(0), inv_t.data_ptr(), scores.data_ptr(),
                             valid.data_ptr(), used.data_ptr(), Nr * m, m, p, k, 1e-12, len(live))
        torch.cuda.synchronize()
    finally:
        native.set_block_inverse_variant("panel")
    assert torch.equal(valid[live], full[2][live])
    # every family sums ||inv|| in a fixed order: the scores are bit-identical too
    assert torch.equal(scores[live], full[1][live])
    assert torch.equal(inv_t[live], full[0][live])
    dead = np.flatnonzero(mine != 0)
    assert torch.equal(valid[dead], sentinel[2][dead]) and torch.equal(inv_t[dead], sentinel[0][dead])


@pytest.mark.parametrize("M,N,K", [(2948, 2900, 520), (2950, 2902, 256), (4096, 2048, 1024)])
@pytest.mark.parametrize("dense", [False, True])
def test_gemm_glds_dense_build(native, M, N, K, dense):
    """The 5-workgroups-per-CU build of the fp64 LDS-DMA trailing update (GemmExtra::dense, the
    engine's choice under a CU reservation) against fp64 torch, with the zero-column / zero-row
    extras and ragged edges, next to the default 4-per-CU build."""
    A = _rand((M, K), torch.float64, 31)
    B = _rand((K, N), torch.float64, 32)
    C = _rand((M, N), torch.float64, 33)
    z0, z1, zr, zh = 128, 384, [0, 1000, 2800], 128
    Cin = C.clone()
    Cin[:, z0:z1] = 0
    for r in zr:
        Cin[r:r + zh] = 0
    ref = Cin + A @ B
    Cd = C.cuda()
    ops.gemm(A.t().contiguous().cuda(), B.cuda(), Cd, op="acc", a_kmajor=True, zero_cols=(z0, z1), zero_rows=zr,
             zero_row_height=zh, dense=dense)
    assert (Cd.cpu() - ref).abs().max().item() < 1e-12 * K


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("variant", ["auto", "narrow"])
@pytest.mark.parametrize("latency", [False, True])
def test_gemm_skip_columns(dtype, variant, latency, native):
    """GemmExtra::skip_c0 / skip_c1 (MAIN's chunk update around the look-ahead columns): the skipped
    output columns keep their bytes, every other column equals the full product bit for bit."""
    M, N, K = 512, 640, 256
    A = _rand((K, M), torch.float64, 61).to(dtype).cuda()
    B = _rand((K, N), torch.float64, 62).to(dtype).cuda()
    C = _rand((M, N), torch.float64, 63).to(dtype).cuda()
    T = torch.full((128, M), 7.0, dtype=dtype, device="cuda") if dtype == torch.float64 else None
    native.set_gemm_variant(variant)
    try:
        full = C.clone()
        Tf = T.clone() if T is not None else None
        ops.gemm(A, B, full, op="acc", a_kmajor=True, latency=latency, tneg=Tf, zero_cols=(64, 192))
        got = C.clone()
        ops.gemm(A, B, got, op="acc", a_kmajor=True, latency=latency, tneg=T, zero_cols=(64, 192),
                 skip_cols=(128, 384))
    finally:
        native.set_gemm_variant("auto")
    keep = torch.zeros(N, dtype=torch.bool, device="cuda")
    keep[128:384] = True
    assert torch.equal(got[:, keep], C[:, keep])
    assert torch.equal(got[:, ~keep], full[:, ~keep])
    if T is not None:  # -C^T of the first 128 columns: outside the skipped range, written
        assert torch.equal(T, Tf)
    with pytest.raises(Exception, match="multiples of 128"):
        ops.gemm(A, B, C.clone(), op="acc", a_kmajor=True, skip_cols=(64, 128))


@pytest.mark.parametrize("shape", [(128, 256, 128), (128, 512, 384), (100, 70, 100), (2048, 128, 256), (128, 96, 5)])
@pytest.mark.parametrize("op", ["acc", "store"])
@pytest.mark.parametrize("extras", ["none", "cin", "tneg", "masks"])
def test_latency_kernel_bit_identical(shape, op, extras, native):
    """gemm_lat_f64 (the register-fed small kernel of the pivot chain's latency launches) against the
    register-staged small tile it replaces: the same products in the same k order, bit for bit,
    including C_in, -C^T, zero row blocks / columns, ragged edges and K not a multiple of 32."""
    M, N, K = shape
    if extras == "cin" and op == "store":
        pytest.skip("C_in is an accumulate-mode input")
    At = _rand((K, M), torch.float64, 71).cuda()
    B = _rand((K, N), torch.float64, 72).cuda()
    C0 = _rand((M, N), torch.float64, 73).cuda()
    kw = {}
    if extras == "cin":
        kw["c_in"] = _rand((M, N), torch.float64, 74).cuda()
    if extras == "masks":
        kw["zero_cols"] = (min(16, N), min(48, N))
        kw["zero_rows"] = (32,)
        kw["zero_row_height"] = 16
    out = []
    for on in (0, 1):
        native.set_lat_kernel(on)
        try:
            C = C0.clone()
            T = torch.full((min(N, 64), M), 3.0, dtype=torch.float64, device="cuda") if extras == "tneg" else None
            ops.gemm(At, B, C, op=op, a_kmajor=True, latency=True, tneg=T, **kw)
            out.append((C, T))
        finally:
            native.set_lat_kernel(-1)
    assert torch.equal(out[0][0], out[1][0])
    if extras == "tneg":
        assert torch.equal(out[0][1], out[1][1])
    cin = (kw.get("c_in", C0)).double().clone()
    if extras == "masks":  # masked entries enter as 0 (GemmExtra zc / zr), the product is still added
        z0, z1 = kw["zero_cols"]
        cin[:, z0:z1] = 0
        for r in kw["zero_rows"]:
            cin[r:r + kw["zero_row_height"]] = 0
    ref = (0 if op == "store" else cin) + At.t() @ B
    # fp64 reference for every case, masks included (the masked case compared the two
    # in-house kernels only)
    assert torch.allclose(out[1][0], ref, rtol=1e-12, atol=1e-10)


def test_latency_batch_kernel_bit_identical(native):
    """gemm_batch on the register-fed tile (GemmExtra::lat_reg) against the small-tile batch: the
    panel-piece products of one pivot step (Store blocks of different K, an Acc block), bit for bit."""
    m = 128
    PP = _rand((3 * m, 4 * m), torch.float64, 81).cuda()
    L = _rand((3 * m, m), torch.float64, 82).cuda()
    out = []
    for on in (0, 1):
        native.set_lat_kernel(on)
        try:
            RP = _rand((m, 4 * m), torch.float64, 83).cuda()
            prods = [("store", L[0:3 * m], PP[0:3 * m, 0:m], RP[:, 0:m]),
                     ("store", L[m:3 * m], PP[m:3 * m, m:2 * m], RP[:, m:2 * m]),
                     ("acc", L[0:3 * m], PP[0:3 * m, 3 * m:4 * m], RP[:, 3 * m:4 * m])]
            ops.gemm_batch(prods)
            out.append(RP)
        finally:
            native.set_lat_kernel(-1)
    assert torch.equal(out[0], out[1])
    ref = L[0:3 * m].t() @ PP[0:3 * m, 0:m]
    assert torch.allclose(out[1][:, 0:m], ref, rtol=1e-12, atol=1e-10)
