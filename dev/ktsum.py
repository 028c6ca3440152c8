"""dev/ktsum.py TAG [passes] -- scatter launches that did a pass (not the exiting clustered/plain
twin) of the last 2 sorts in gpurun_out/kt_TAG, in order, and their per-pass means."""
import csv, glob, sys
import os
f = max(glob.glob(f"gpurun_out/kt_{sys.argv[1]}/*/*kernel_trace.csv"), key=os.path.getmtime)
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if "rs_scatter" in r["Kernel_Name"]]
d = [x for x in d if x > 0.1 * max(d)][-2 * P:]
print(sys.argv[1], " ".join(f"{x:.3f}" for x in d), "| per pass", " ".join(f"{(d[i] + d[i + P]) / 2:.3f}" for i in range(P)))
