#!/usr/bin/env python3
"""Per-call time of the pivot chain's small GEMMs (``latency=True`` launches), back to back on one
stream on an otherwise idle GPU: the floor the in-solve times (rocprofv3 traces) compare against.

    python bench/lat_gemm_probe.py [--reps R] [--shapes M,N,K ...] [--tneg]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpi_jordan_crazy_acceleration_amd import load_native, ops  # noqa: E402

# column updates (rows x m x j*m), panel pieces (m x d*m x m), look-ahead rows / chunk pass
DEFAULT = ["2048,128,128", "2048,128,256", "2048,128,384", "4096,128,384", "8192,128,128", "16384,128,384",
           "128,512,128", "128,512,384", "128,4096,384", "128,8192,128"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--shapes", nargs="*", default=DEFAULT)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    load_native()
    for s in a.shapes:
        M, N, K = (int(x) for x in s.split(","))
        At = torch.randn(K, M, dtype=torch.float64, device="cuda")
        B = torch.randn(K, N, dtype=torch.float64, device="cuda")
        C = torch.randn(M, N, dtype=torch.float64, device="cuda")
        tn = torch.empty(min(N, 128), M, dtype=torch.float64, device="cuda")
        err = None
        if a.check:
            C0 = C.clone()
            ops.gemm(At, B, C, op="acc", a_kmajor=True, latency=True, tneg=tn)
            ref = C0 + At.t() @ B
            err = float((C - ref).abs().max() / ref.abs().max())
            err = max(err, float((tn + ref[:, :tn.shape[0]].t()).abs().max() / ref.abs().max()))
        for _ in range(5):
            ops.gemm(At, B, C, op="acc", a_kmajor=True, latency=True, tneg=tn)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ops.gemm(At, B, C, op="acc", a_kmajor=True, latency=True, tneg=tn)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.reps * 1e6
        print(json.dumps({"M": M, "N": N, "K": K, "us_per_call": round(us, 2),
                          "tflops": round(2.0 * M * N * K / us / 1e6, 2), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
