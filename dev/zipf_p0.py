"""dev/zipf_p0.py -- why is pass 0 of the Zipf-keys sort slower in bench.py (2.36 ms) than in
dev/lines_exp (1.75 ms)? Times the library's pass-0 scatter on the same keys in several contexts."""
import sys, time
from pathlib import Path
import numpy as np
import torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import radixsort as rs
from _util import zipf_cdf_u32

n = 1 << 30
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
keys = rs.empty_u32(n, dev)
dist = sys.argv[1] if len(sys.argv) > 1 else "zipf"
if dist == "zipf":
    rs.gen_zipf(keys, rs.from_numpy_u32(zipf_cdf_u32(), dev), 0x5EED)
else:
    rs.gen_uniform(keys, 0x5EED)
p = rs.plan(n, 8, False, 0)
print("plan", p.num_chunks, p.tiles_per_chunk, p.tile_keys, flush=True)
table = torch.empty(p.table_entries, dtype=torch.int32, device=dev)
bs = torch.empty(max(1, p.scan_blocks), dtype=torch.int32, device=dev)
out = rs.empty_u32(n, dev)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return np.median(ts)


for shift in (0, 8, 16, 24):
    rs.pass_histogram(p, keys, shift, table)
    rs.pass_scan(p, table, bs)
    t = timed(lambda: rs.pass_scatter(p, keys, out, shift, table))
    print(f"{dist} scatter shift={shift} on the raw keys: {t:.3f} ms", flush=True)
# the full sort, per phase
ws = rs.workspace(p.workspace_bytes, dev)
with rs.Profile() as prof:
    for _ in range(3):
        rs.sort_device(keys, out, 8, ws=ws, plan_=p)
    torch.cuda.synchronize()
print(dist, "sort phases", {k: (round(v["ms"] / 3, 3), v["launches"]) for k, v in prof.times.items()}, flush=True)
# pass 0 in isolation, into different destinations, after the plain and the joint histogram
tmpk = ws[: n * 4].view(torch.int32)  # the workspace's ping-pong buffer (where a 4-pass sort's pass 0 writes)
other = rs.empty_u32(n, dev)
rs.pass_histogram(p, keys, 0, table)
rs.pass_scan(p, table, bs)
for name, dst in (("out", out), ("ws tmp_k", tmpk), ("fresh", other)):
    t = timed(lambda: rs.pass_scatter(p, keys, dst, 0, table))
    print(f"{dist} pass-0 scatter into {name}: {t:.3f} ms", flush=True)
