#!/usr/bin/env python3
"""Latency of the batched candidate-block inversion (pivot search) in isolation (device-side events).

    [BI_M="64 128"] [BI_NBLK="8 32 64 256"] [BI_REPS=50] python bench/bench_blockinv.py [panel] [sweep] [co] [generic] [huge]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpi_jordan_crazy_acceleration_amd import load_native, ops  # noqa: E402


def main(variants):
    C = load_native()
    for var in variants:
        C.set_block_inverse_variant(var)
        for m in [int(x) for x in os.environ.get("BI_M", "64 128").split()]:
            for nblk in [int(x) for x in os.environ.get("BI_NBLK", "8 32 64 256").split()]:
                for dt in (torch.float64, torch.float32):
                    Lt = torch.randn(m, nblk * m, dtype=dt, device="cuda")
                    n = nblk * m
                    inv_t, scores, valid = ops.block_inverse(Lt, n, m)
                    used = torch.zeros(nblk, dtype=torch.int32, device="cuda")
                    torch.cuda.synchronize()
                    # device-side: 50 back-to-back launches between two events
                    us = ops.device_for(Lt).time_block_inverse(
                        ops._DT[dt], Lt.data_ptr(), Lt.stride(0), inv_t.data_ptr(), scores.data_ptr(),
                        valid.data_ptr(), used.data_ptr(), n, m, 1, 0, 0.0, int(os.environ.get("BI_REPS", "50")))
                    print(json.dumps({"variant": var, "m": m, "nblk": nblk, "dtype": str(dt).split(".")[-1],
                                      "us_per_call": round(us, 1), "us_per_step": round(us / m, 3)}), flush=True)
    C.set_block_inverse_variant("panel")


if __name__ == "__main__":
    main(sys.argv[1:] or ["panel", "sweep"])
