#!/usr/bin/env python3
"""Reduce scripts/smi_sample.py output to a clock / power / temperature table.

    python3 scripts/smi_summary.py gpurun_out/sus/smi_32768.jsonl [--every 2]

One row per sample (or every k-th): time, mean and min/max shader clock over the XCDs, socket power,
hotspot temperature, gfx activity; then the same averaged over the busy samples (gfx activity >= 90).
"""
from __future__ import annotations

import json
import sys


def rows(path):
    for line in open(path):
        s = json.loads(line)
        raw = s.get("raw")
        if not raw:
            continue
        g = raw["gpu_data"][0] if isinstance(raw, dict) else raw[0]
        clks = [v["clk"]["value"] for k, v in g.get("clock", {}).items()
                if k.startswith("gfx_") and isinstance(v.get("clk"), dict)]
        pw = g.get("power", {}).get("socket_power", {})
        tmp = g.get("temperature", {}).get("hotspot", {})
        act = g.get("usage", {}).get("gfx_activity", {})
        yield {"t": s["t"], "clk_mean": sum(clks) / len(clks) if clks else None,
               "clk_min": min(clks) if clks else None, "clk_max": max(clks) if clks else None,
               "power_w": pw.get("value") if isinstance(pw, dict) else None,
               "hotspot_c": tmp.get("value") if isinstance(tmp, dict) else None,
               "gfx_pct": act.get("value") if isinstance(act, dict) else None}


def main(argv):
    path = argv[0]
    every = int(argv[argv.index("--every") + 1]) if "--every" in argv else 1
    rs = list(rows(path))
    print("| t (s) | gfx clock MHz mean [min-max over XCDs] | socket W | hotspot °C | gfx % |")
    print("|---|---|---|---|---|")
    for i, r in enumerate(rs):
        if i % every:
            continue
        print(f"| {r['t']:.1f} | {r['clk_mean']:.0f} [{r['clk_min']}-{r['clk_max']}] | {r['power_w']} | "
              f"{r['hotspot_c']} | {r['gfx_pct']} |")
    busy = [r for r in rs if (r["gfx_pct"] or 0) >= 90]
    if busy:
        n = len(busy)
        print(f"\nbusy samples (gfx >= 90 %): {n}; clock mean {sum(r['clk_mean'] for r in busy) / n:.0f} MHz "
              f"(min sample {min(r['clk_mean'] for r in busy):.0f}, max {max(r['clk_mean'] for r in busy):.0f}); "
              f"power mean {sum(r['power_w'] for r in busy) / n:.0f} W (max {max(r['power_w'] for r in busy)}); "
              f"hotspot {min(r['hotspot_c'] for r in busy)}-{max(r['hotspot_c'] for r in busy)} °C")


if __name__ == "__main__":
    main(sys.argv[1:])
