"""dev/ktall.py TAG [count] -- the last `count` kernel launches of gpurun_out/kt_TAG in order:
duration, gap before it, short name."""
import csv, glob, os, re, sys
f = max(glob.glob(f"gpurun_out/kt_{sys.argv[1]}/*/*kernel_trace.csv"), key=os.path.getmtime)
N = int(sys.argv[2]) if len(sys.argv) > 2 else 24
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-N:]
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"void rsort::|\(.*", "", r["Kernel_Name"])[:70]
    print(f"{(e - s) / 1e6:8.4f} ms  gap {((s - prev) / 1e6 if prev else 0):7.4f}  {name}")
    prev = e
