#!/usr/bin/env python3
"""torch.addmm (hipBLASLt / rocBLAS) at one trailing-update shape, for rocprofv3 counter passes
next to bench/gemm_probe.py (the solver's own kernel): C += A B, M x N x K, fp64, A row-major
(--kmajor: A stored K-major as the solver keeps its multipliers, passed transposed).

    python bench/vendor_probe.py [M N K] [--kmajor] [--reps R]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", nargs="*", type=int, default=[32768, 8192, 512])
    ap.add_argument("--kmajor", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    M, N, K = a.shape
    A = torch.randn(K, M, dtype=torch.float64, device="cuda").t() if a.kmajor else \
        torch.randn(M, K, dtype=torch.float64, device="cuda")
    B = torch.randn(K, N, dtype=torch.float64, device="cuda")
    C = torch.randn(M, N, dtype=torch.float64, device="cuda")
    C.addmm_(A, B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        C.addmm_(A, B)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(json.dumps({"M": M, "N": N, "K": K, "library": "torch.addmm", "a_kmajor": a.kmajor,
                      "ms": round(dt * 1e3, 4), "tflops": round(2.0 * M * N * K / dt / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
