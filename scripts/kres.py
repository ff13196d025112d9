#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin): one line per kernel."""
import re, sys, subprocess
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    kv = m.group(1)
    if kv.startswith("Function Name:"):
        cur = {"name": kv.split(":", 1)[1].strip()}; rows.append(cur); continue
    if cur is None or ":" not in kv: continue
    k, v = kv.split(":", 1); cur[k.strip()] = v.strip()
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat not in r["name"]: continue
    try: dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    except Exception: dem = r["name"]
    dem = re.sub(r"gj::kern::", "", dem)
    print(f'{r.get("VGPRs","?"):>4} v {r.get("AGPRs","?"):>3} a spill {r.get("VGPRs Spill","?"):>4} occ {r.get("Occupancy [waves/SIMD]","?")} lds {r.get("LDS Size [bytes/block]","?"):>6}  {dem[:150]}')
