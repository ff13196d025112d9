#!/usr/bin/env python3
"""RCCL kernels in rocprofv3 (rocpd sqlite) kernel traces: grid, workgroup size, LDS, VGPRs and
duration per kernel name -- the CU footprint of a collective, for ShadowComm's cost model
(shadow_comm.cpp spin workgroups).  Usage: rccl_footprint.py <db> [<db> ...]"""
import collections
import sqlite3
import sys


def main(dbs):
    agg = collections.defaultdict(lambda: [0, 0.0, set(), set(), set(), set()])
    for db in dbs:
        con = sqlite3.connect(db)
        for name, gx, wx, dur, vgpr, agpr, lds in con.execute(
                "select name, grid_x, workgroup_x, duration, vgpr_count, accum_vgpr_count, lds_size from kernels"):
            low = name.lower()
            if "nccl" not in low and "rccl" not in low:
                continue
            k = name.split("(")[0][:80]
            a = agg[k]
            a[0] += 1
            a[1] += dur
            a[2].add(gx // max(wx, 1))
            a[3].add(wx)
            a[4].add(lds)
            a[5].add((vgpr, agpr))
    print("| RCCL kernel | calls | avg us | workgroups | threads / WG | LDS B | VGPR, AGPR |")
    print("|---|---|---|---|---|---|---|")
    for k, a in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"| `{k}` | {a[0]} | {a[1] / a[0] / 1e3:.1f} | {sorted(a[2])} | {sorted(a[3])} | {sorted(a[4])} | "
              f"{sorted(a[5])} |")


if __name__ == "__main__":
    main(sys.argv[1:])
