#!/usr/bin/env python3
"""Idle gaps of the trailing-update (MAIN) stream in the LAST solve of a rocprofv3 kernel trace:
total idle, the gap histogram, and for the largest gaps which kernel ran last on every other
stream (what MAIN was most likely waiting for).

    python scripts/main_gaps.py gpurun_out/prof_x/run_results.db
"""
import collections
import sqlite3
import sys


def short(name):
    n = name.split("(")[0]
    for key in ("block_inverse", "pivot_select", "pivot_local", "pivot_global", "owner_edits", "gemm_batch",
                "extract", "h_block", "gemm_glds", "gemm_kernel", "spin_kernel", "copyBuffer", "fillBuffer",
                "generate", "permute"):
        if key in n:
            return key
    return n[-40:]


def main(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    # MAIN = the stream with the most gemm_glds time
    busy = collections.Counter()
    for r in rows:
        if "gemm_glds" in r[0] or "gemm_kernel" in r[0]:
            busy[r[3]] += r[2] - r[1]
    main_s = busy.most_common(1)[0][0]
    gens = [r for r in rows if "generate" in r[0]]
    t0 = gens[-1][2] if gens else rows[0][1]  # last solve starts after its generate
    perm = [r for r in rows if "permute" in r[0] and r[1] > t0]
    t1 = perm[-1][2] if perm else rows[-1][2]
    mrows = [r for r in rows if r[3] == main_s and t0 <= r[1] <= t1]
    gaps = []
    for a, b in zip(mrows, mrows[1:]):
        g = b[1] - a[2]
        if g > 0:
            gaps.append((g, a, b))
    span = (t1 - t0) / 1e6
    idle = sum(g for g, _, _ in gaps) / 1e6
    print(f"MAIN stream {main_s}: span {span:.2f} ms, busy {span - idle:.2f} ms, idle {idle:.2f} ms "
          f"({100 * idle / span:.1f} %) in {len(gaps)} gaps\n")
    hist = collections.Counter()
    for g, _, _ in gaps:
        us = g / 1e3
        hist["<5 us" if us < 5 else "5-20 us" if us < 20 else "20-100 us" if us < 100 else "100-500 us" if us < 500 else ">=500 us"] += us
    print("| gap size | total ms |\n|---|---|")
    for k in ("<5 us", "5-20 us", "20-100 us", "100-500 us", ">=500 us"):
        print(f"| {k} | {hist[k] / 1e3:.2f} |")
    print("\nLargest gaps (what ran last on the other streams before MAIN resumed):\n")
    print("| gap us | MAIN before -> after | last kernels ending before resume on other streams |")
    print("|---|---|---|")
    for g, a, b in sorted(gaps, reverse=True)[:12]:
        last = {}
        for r in rows:
            if r[3] != main_s and r[2] <= b[1] and r[2] >= a[2]:
                last[r[3]] = short(r[0])
        print(f"| {g / 1e3:.0f} | {short(a[0])} -> {short(b[0])} | {', '.join(f's{s}:{k}' for s, k in sorted(last.items()))} |")


if __name__ == "__main__":
    main(sys.argv[1])
