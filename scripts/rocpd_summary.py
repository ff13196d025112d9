#!/usr/bin/env python3
"""Summarise a rocprofv3 (rocpd sqlite) kernel trace: top kernels and per-stream busy/idle time."""
import collections
import sqlite3
import sys


def main(db, title=""):
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = cur.execute("select name, grid_x/workgroup_x, duration, start, end, stream_id, vgpr_count, "
                       "accum_vgpr_count, lds_size from kernels order by start").fetchall()
    print(f"# rocprofv3 kernel-trace summary {title}\n")
    print(f"source: `{db}` ({len(rows)} dispatches)\n")
    agg = collections.defaultdict(lambda: [0, 0.0, 0, 0, 0])
    for r in rows:
        k = (r[0].split("(")[0][:90], r[1])
        a = agg[k]
        a[0] += 1
        a[1] += r[2]
        a[2], a[3], a[4] = r[6], r[7], r[8]
    tot = sum(v[1] for v in agg.values())
    print("| kernel | workgroups | calls | total ms | avg us | % | VGPR | AGPR | LDS B |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (name, grid), v in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print(f"| `{name}` | {grid} | {v[0]} | {v[1]/1e6:.2f} | {v[1]/v[0]/1e3:.1f} | {100*v[1]/tot:.1f} | {v[2]} | {v[3]} | {v[4]} |")
    span = (rows[-1][4] - rows[0][3]) / 1e6 if rows else 0
    print(f"\ntrace span: {span:.1f} ms\n")
    print("| stream | kernels | busy ms | busy % of span |")
    print("|---|---|---|---|")
    by = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        by[r[5]][0] += 1
        by[r[5]][1] += r[2]
    for s, v in sorted(by.items()):
        print(f"| {s} | {v[0]} | {v[1]/1e6:.1f} | {100*v[1]/1e6/span:.1f} |")
    print("\n## By kernel (all grid sizes together)\n")
    print("| kernel | streams | calls | total ms | avg us | workgroups per call | % |")
    print("|---|---|---|---|---|---|---|")
    kn = collections.defaultdict(lambda: [0, 0.0, 0, set()])
    for r in rows:
        a = kn[r[0].split("(")[0][:70]]
        a[0] += 1
        a[1] += r[2]
        a[2] += r[1]
        a[3].add(r[5])
    for name, v in sorted(kn.items(), key=lambda x: -x[1][1])[:16]:
        st = ",".join(str(x) for x in sorted(v[3]))
        print(f"| `{name}` | {st} | {v[0]} | {v[1]/1e6:.2f} | {v[1]/v[0]/1e3:.1f} | {v[2]/v[0]:.1f} | {100*v[1]/tot:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
