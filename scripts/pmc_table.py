#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counter CSVs (counter_collection.csv files under a directory),
for the dominant kernel of each pass directory: `python3 scripts/pmc_table.py gpurun_out/stall`."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    rows = defaultdict(lambda: defaultdict(list))  # (who, kernel) -> counter -> values
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        who = os.path.relpath(path, root).split(os.sep)[0].rsplit("_p", 1)[0]
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "?")
                rows[(who, k)][r.get("Counter_Name", "?")].append(float(r.get("Counter_Value", "nan")))
    # the kernel with the most dispatches per source is the GEMM under test
    best = {}
    for (who, k), ctr in rows.items():
        n = max(len(v) for v in ctr.values())
        if who not in best or n > best[who][1]:
            best[who] = (k, n)
    names = sorted({c for (who, k), ctr in rows.items() if best.get(who, (None,))[0] == k for c in ctr})
    print("| counter | " + " | ".join(f"{w}: {best[w][0][:48]}" for w in sorted(best)) + " |")
    print("|---|" + "---|" * len(best))
    for c in names:
        vals = []
        for w in sorted(best):
            v = rows[(w, best[w][0])].get(c, [])
            vals.append(f"{sum(v) / len(v):.4g}" if v else "-")
        print(f"| {c} | " + " | ".join(vals) + " |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stall")
