#!/usr/bin/env python3
"""Vendor-library reference point for the trailing-update GEMM: torch.addmm (rocBLAS / hipBLASLt)
at the solver's shapes, fp64, C += A B — next to this framework's LDS-DMA MFMA kernel
(bench/gemm_probe.py).  Device-side timing, 20 back-to-back calls.

    python bench/bench_vendor_gemm.py
"""
import json

import torch


def main():
    shapes = [(32768, 4096, 512), (32768, 8192, 512), (4096, 32768, 1024), (16384, 8192, 512)]
    for M, N, K in shapes:
        for dt, kmajor in ((torch.float64, False), (torch.float64, True), (torch.float32, False)):
            # kmajor: A stored K-major (K x M contiguous, the solver's multiplier panel) -> At.t()
            A = (torch.randn(K, M, dtype=dt, device="cuda").t() if kmajor
                 else torch.randn(M, K, dtype=dt, device="cuda"))
            B = torch.randn(K, N, dtype=dt, device="cuda")
            C = torch.randn(M, N, dtype=dt, device="cuda")
            for _ in range(3):
                C.addmm_(A, B)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                C.addmm_(A, B)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(json.dumps({"M": M, "N": N, "K": K, "dtype": str(dt).split(".")[-1], "library": "torch.addmm",
                              "a_layout": "k-major" if kmajor else "row-major",
                              "ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9, 2)}), flush=True)
            del A, B, C


if __name__ == "__main__":
    main()
