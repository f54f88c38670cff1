#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a hipcc --save-temps .s file.
usage: isa_hist.py FILE.s KERNEL_SUBSTRING"""
import collections, re, sys
src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
inside = False; hist = collections.Counter(); labels = []
for ln in lines:
    if not inside:
        if re.match(r"^\S*%s\S*:\s*(;.*)?$" % re.escape(pat), ln) and not ln.startswith("."):
            inside = True
        continue
    if ln.startswith("\t.end_amdhsa") or re.match(r"^\.Lfunc_end", ln):
        break
    s = ln.strip()
    if not s or s.startswith(";") or s.startswith("."):
        if re.match(r"^\.LBB", s): labels.append(s)
        continue
    op = s.split()[0]
    hist[op] += 1
tot = sum(hist.values())
cls = collections.Counter()
for op, n in hist.items():
    c = ("valu-mul" if re.match(r"v_(mul|mad)", op) else "valu" if op.startswith("v_") else
         "lds" if op.startswith("ds_") else "vmem" if op.startswith(("buffer_", "global_")) else
         "smem" if op.startswith("s_load") or op.startswith("s_buffer") else "salu" if op.startswith("s_") else "other")
    cls[c] += n
print("total", tot, dict(cls), "blocks", len(labels))
for op, n in hist.most_common(40): print(f"{n:7d} {op}")
