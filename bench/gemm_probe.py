#!/usr/bin/env python3
"""Single-shape GEMM probe for rocprofv3 counter passes (one kernel shape, fixed repetitions).

    python bench/gemm_probe.py [M N K] [--dtype fp64|fp32] [--variant narrow|big|bigpf|squarepf|glds|auto] [--reps R]

Prints one JSON line with the achieved rate; meant to run under
``rocprofv3 --pmc <counters> -- python3 bench/gemm_probe.py ...``.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpi_jordan_crazy_acceleration_amd import load_native, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", nargs="*", type=int, default=[32768, 4096, 512])
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--variant", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--check", action="store_true", help="compare one call against torch fp64")
    ap.add_argument("--op", default="acc", choices=["acc", "store"], help="C += A B or C = A B")
    ap.add_argument("--lda", type=int, default=0, help="row stride of A^T (default M)")
    ap.add_argument("--ldb", type=int, default=0, help="row stride of B (default N)")
    ap.add_argument("--ldc", type=int, default=0, help="row stride of C (default N; the solver's is the padded order)")
    a = ap.parse_args()
    M, N, K = a.shape
    C_ = load_native()
    if a.variant:
        C_.set_gemm_variant(a.variant)
    dt = torch.float64 if a.dtype == "fp64" else torch.float32
    At = torch.randn(K, max(a.lda, M), dtype=dt, device="cuda")[:, :M]
    B = torch.randn(K, max(a.ldb, N), dtype=dt, device="cuda")[:, :N]
    C = torch.randn(M, max(a.ldc, N), dtype=dt, device="cuda")[:, :N]
    err = None
    if a.check:
        C0 = C.clone()
        ops.gemm(At, B, C, op="acc", a_kmajor=True)
        ref = C0.double() + At.double().t() @ B.double()
        err = float((C.double() - ref).abs().max() / ref.abs().max())
        del C0, ref
    ops.gemm(At, B, C, op=a.op, a_kmajor=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ops.gemm(At, B, C, op=a.op, a_kmajor=True)
    torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / a.reps
    print(json.dumps({"M": M, "N": N, "K": K, "dtype": a.dtype, "variant": a.variant or "default", "op": a.op,
                      "lda": At.stride(0), "ldb": B.stride(0), "ldc": C.stride(0),
                      "ms": round(dt_s * 1e3, 4), "tflops": round(2.0 * M * N * K / dt_s / 1e12, 2), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
