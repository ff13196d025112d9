#!/usr/bin/env python3
"""Microbenchmark of the elimination GEMM kernel (C += A^T-stored * B) at the solver's shapes."""
import json
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpi_jordan_crazy_acceleration_amd import ops  # noqa: E402


def run(M, N, K, dtype, reps=10):
    At = torch.randn(K, M, dtype=dtype, device="cuda")
    B = torch.randn(K, N, dtype=dtype, device="cuda")
    C = torch.randn(M, N, dtype=dtype, device="cuda")
    ops.gemm(At, B, C, op="acc", a_kmajor=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.gemm(At, B, C, op="acc", a_kmajor=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    tf = 2.0 * M * N * K / dt / 1e12
    bw = 2.0 * M * N * C.element_size() / dt / 1e12
    return {"M": M, "N": N, "K": K, "dtype": str(dtype).split(".")[-1], "ms": round(dt * 1e3, 3),
            "tflops": round(tf, 2), "c_rw_TBps": round(bw, 2)}


if __name__ == "__main__":
    from mpi_jordan_crazy_acceleration_amd import load_native
    C = load_native()
    variants = sys.argv[1:] or ["big"]
    for v in variants:
        C.set_gemm_variant(v)
        for dt in (torch.float64, torch.float32):
            for (M, N, K) in [(32768, 4096, 128), (32768, 4096, 256), (4096, 4096, 128), (32768, 128, 128)]:
                if v == "valu" and dt == torch.float32:
                    continue
                r = run(M, N, K, dt)
                r["variant"] = v
                print(json.dumps(r), flush=True)
