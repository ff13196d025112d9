#!/usr/bin/env python3
"""Policy-cliff sweep: for each N, the engine's auto policy against its
neighbours -- CU reservation flipped (0 <-> 32), depth flipped (2 <-> 4), and the skip_cols / lat_reg
pair flipped -- on one GPU, fp64, m = 128, each a `bench.py` run (subprocess) with the override in
its environment.  Writes one JSON line per run to OUT and prints a markdown table.

    python3 scripts/policy_sweep.py OUT.jsonl [--sizes 6144,12288,20480,24576,40960] [--steps 5 --warmup 2]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(n, env_extra, steps, warmup, timeout):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--size", str(n), "--steps", str(steps),
                        "--warmup", str(warmup)], env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise SystemExit(f"bench.py N={n} {env_extra} failed rc={r.returncode}: {r.stderr[-1500:]}")
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--sizes", default="6144,12288,20480,24576,40960")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=240)
    a = ap.parse_args()
    rows = []
    with open(a.out, "a") as f:
        for n in [int(x) for x in a.sizes.split(",")]:
            base = run(n, {}, a.steps, a.warmup, a.timeout)
            pol = base["policy"]
            variants = [("auto", {})]
            variants.append((f"reserve {32 if pol['reserve_cus'] == 0 else 0}",
                             {"GJ_RESERVE_CUS": "32" if pol["reserve_cus"] == 0 else "0"}))
            variants.append((f"depth {2 if pol['depth'] != 2 else 4}", {}))
            flip = "0" if pol["skip_cols"] else "1"
            variants.append((f"skip_cols+lat_reg {flip}",
                             {"GJ_SKIP_COLS": flip, "GJ_CHUNK_SKIP": flip, "GJ_LAT_REG": flip}))
            for name, env in variants:
                if name == "auto":
                    d = base
                elif name.startswith("depth"):
                    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--size", str(n),
                                        "--steps", str(a.steps), "--warmup", str(a.warmup), "--depth",
                                        name.split()[1]], capture_output=True, text=True, timeout=a.timeout)
                    if r.returncode != 0:
                        raise SystemExit(f"depth run failed: {r.stderr[-1500:]}")
                    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
                else:
                    d = run(n, env, a.steps, a.warmup, a.timeout)
                rec = {"n": n, "variant": name, "env": env, "ms": d["ms_per_step"], "tflops": d["value"] / 1e3,
                       "check": d["check"], "policy": d["policy"], "step_ms": d.get("step_ms")}
                f.write(json.dumps(rec) + "\n")
                f.flush()
                rows.append(rec)
                print(f"N={n} {name}: {d['ms_per_step']:.2f} ms ({d['value'] / 1e3:.1f} TF/s) {d['check']}",
                      flush=True)
    print("\n| N | variant | ms / inversion | TF/s | vs auto |")
    print("|---|---|---|---|---|")
    for r in rows:
        auto = next(x for x in rows if x["n"] == r["n"] and x["variant"] == "auto")
        print(f"| {r['n']} | {r['variant']} | {r['ms']:.2f} | {r['tflops']:.1f} | {r['ms'] / auto['ms'] - 1:+.1%} |")


if __name__ == "__main__":
    main()
