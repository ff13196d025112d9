#!/usr/bin/env python3
"""Critical-path view of the pivot chain from a rocprofv3 kernel trace (rocpd sqlite).

For the stream that runs the candidate-block inverses (SIDE), split the last solve into steps at
each block-inverse dispatch and report, per kernel kind, the mean time per step spent executing
and the mean idle gap before it (waiting for the host's enqueue, for an event of another stream,
or for free CUs).  The sum is the per-step chain length.

    python scripts/side_chain.py gpurun_out/prof_x/run_results.db [steps [depth]]
"""
import collections
import sqlite3
import sys


def short(name):
    n = name.split("(")[0]
    for key in ("block_inverse", "pivot_select", "pivot_local", "pivot_global", "owner_edits",
                "gemm_batch", "extract", "h_block", "gemm_glds", "gemm_kernel", "copyBuffer", "fillBuffer"):
        if key in n:
            return key
    return n[-40:]


def main(db, nsteps=None, depth=0):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end, stream_id, grid_x/workgroup_x from kernels order by start").fetchall()
    bi = [r for r in rows if "block_inverse" in r[0]]
    side = bi[-1][3]
    srows = [r for r in rows if r[3] == side]
    starts = [r[1] for r in srows if "block_inverse" in r[0]]
    # the last solve: steps are the last nsteps block-inverse dispatches (default: all after the last big gap)
    if nsteps is None:
        gaps = [b - a for a, b in zip(starts, starts[1:])]
        big = max(range(len(gaps)), key=lambda i: gaps[i]) if gaps else -1
        starts = starts[big + 1:]
    else:
        starts = starts[-nsteps:]
    t0, t1 = starts[0], srows[-1][2]
    sel = [r for r in srows if t0 <= r[1] <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    prev_end = None
    for r in sel:
        k = short(r[0])
        a = agg[k]
        a[0] += 1
        a[1] += (r[2] - r[1]) / 1e3
        if prev_end is not None:
            a[2] += max(0.0, (r[1] - prev_end) / 1e3)
        prev_end = r[2]
    n = len(starts)
    print(f"SIDE stream {side}: {n} steps over {(t1 - t0) / 1e6:.2f} ms ({(t1 - t0) / 1e3 / n:.1f} us per step)\n")
    print("| kernel | calls/step | busy us/step | idle-before us/step |")
    print("|---|---|---|---|")
    tb = tg = 0.0
    for k, a in sorted(agg.items(), key=lambda x: -(x[1][1] + x[1][2])):
        print(f"| {k} | {a[0] / n:.2f} | {a[1] / n:.1f} | {a[2] / n:.1f} |")
        tb += a[1]
        tg += a[2]
    print(f"| **total** | | **{tb / n:.1f}** | **{tg / n:.1f}** |")
    if depth:
        # wait before each step's block inverse, by the step's position in its panel (position 0
        # waits for MAIN's look-ahead update, later ones only for this stream's own work)
        pos = collections.defaultdict(list)
        prev = None
        for r in sel:
            if "block_inverse" in r[0] and prev is not None:
                i = starts.index(r[1]) if r[1] in starts else None
                if i is not None:
                    pos[i % depth].append((r[1] - prev) / 1e3)
            prev = r[2]
        print("\n| step in panel | idle before block_inverse, mean us |")
        print("|---|---|")
        for j in sorted(pos):
            print(f"| {j} | {sum(pos[j]) / len(pos[j]):.1f} |")
    others = collections.defaultdict(float)
    for r in rows:
        if r[3] != side and t0 <= r[1] <= t1:
            others[r[3]] += (min(r[2], t1) - r[1]) / 1e3
    for s, v in sorted(others.items()):
        print(f"\nstream {s}: busy {v / 1e3:.2f} ms of {(t1 - t0) / 1e6:.2f} ms ({100 * v * 1e3 / (t1 - t0):.0f} %)", end="")
    print()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None, int(sys.argv[3]) if len(sys.argv) > 3 else 0)
