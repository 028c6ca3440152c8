"""Instruction counts of one kernel between its barriers (the .s of a --save-temps build):
python dev/isa_phases.py file.s 'mangled-name-substring'"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
seg, segs = Counter(), []
names = []
for l in body:
    s = l.strip()
    if not s or s.startswith((";", ".")) or s.endswith(":"):
        if s.startswith(".LBB"):
            seg["#blocks"] += 1
        continue
    op = s.split()[0]
    cls = ("ds_" if op.startswith("ds_") else "global" if op.startswith(("global_", "buffer_")) else
           "s_wait" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else "valu")
    seg[cls] += 1
    seg["total"] += 1
    if op == "s_barrier":
        segs.append(seg)
        seg = Counter()
segs.append(seg)
for i, c in enumerate(segs):
    print(i, dict(c))
