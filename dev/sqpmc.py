"""Summarise `dev/lab.sh sqpmc`: per kernel symbol, the mean of each SQ counter over its dispatches, and
the cycle shares (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_* over SQ_WAVE_CYCLES; all count
quad-cycles per wave). python dev/sqpmc.py gpurun_out"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
if len(sys.argv) > 3 and sys.argv[2] == "--order":
    # every working scatter dispatch of the run in issue order, one row each
    rows = defaultdict(dict)
    for f in (root / sys.argv[3] if (root / sys.argv[3]).is_dir() else root).rglob("*counter_collection.csv"):
        if sys.argv[3] not in str(f):
            continue
        for r in csv.DictReader(open(f)):
            if "rs_scatter" in r["Kernel_Name"]:
                rows[(int(r["Dispatch_Id"]), r["Kernel_Name"])][r["Counter_Name"]] = float(r["Counter_Value"])
    names = None
    for (did, kn), cs in sorted(rows.items()):
        if cs.get("SQ_WAVE_CYCLES", 0) < 1e6:
            continue
        names = names or sorted(cs)
        print(did, kn.split("(")[0].replace("void rsort::", "")[-12:], " ".join(f"{c[3:]}={cs[c]:.3g}" for c in names))
    sys.exit(0)
for prog in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("pairs", "keys")):
    agg = defaultdict(lambda: defaultdict(list))
    for d in sorted(root.glob(f"sqpmc_{prog}_*")):
        if not d.is_dir():
            continue
        for f in d.rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                kn = r["Kernel_Name"]
                if "rs_scatter" not in kn:
                    continue
                agg[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kn, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0)
        if wc < 1e6:  # (the unselected twin that exits at once)
            continue
        print(f"== {prog}: {kn[:110]}")
        for c in sorted(m):
            extra = f"  ({m[c] / wc:.3f} of wave cycles)" if wc and (c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE")) else ""
            print(f"   {c:32s} {m[c]:16.4g}{extra}")
