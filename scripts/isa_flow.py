#!/usr/bin/env python3
"""Compress a kernel's ISA (hipcc -S output) into its load/wait/barrier/MFMA flow.

    isa_flow.py file.s <mangled-symbol-substring>
"""
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name)
i = s.index(":", i)
j = s.index(".Lfunc_end", i)
out = []
for line in s[i:j].splitlines():
    t = line.strip()
    if t.startswith(("s_waitcnt", "s_barrier", "s_cbranch", ".LBB")):
        out.append(t.split(";")[0].strip())
    elif "mfma" in t:
        out.append("MFMA")
    elif t.startswith("buffer_load"):
        out.append("BL")
    elif t.startswith("buffer_store"):
        out.append("BS")
    elif t.startswith("ds_write"):
        out.append("DSW")
    elif t.startswith("ds_read"):
        out.append("DSR")
    elif "scratch_" in t:
        out.append("SCRATCH")
comp, prev, cnt = [], None, 0
for o in out + [None]:
    if o == prev:
        cnt += 1
        continue
    if prev:
        comp.append(f"{prev}x{cnt}" if cnt > 1 else prev)
    prev, cnt = o, 1
print("\n".join(comp))
