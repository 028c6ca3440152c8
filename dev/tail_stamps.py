# Backs DESIGN §3 tail_scan row: the timeline of a tail-scanned C2 pass (s_memrealtime stamps).
"""dev/tail_stamps.py -- with the stamps variant of the library (dev/build_variant.sh tstamp2 ...), the
timeline of the last tail-scanned pass at C2 (s_memrealtime, 100 MHz): first workgroup start, last
workgroup's end of work, tail start, tail end."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cuda.radixsort_amd"))
import torch
import radixsort as rs
n, k = 1 << 26, 4
x = torch.empty(n, dtype=torch.int32, device="cuda")
rs.gen_uniform(x, 0x5EED)
y = torch.empty_like(x)
p = rs.plan(n, k)
ws = rs.workspace(p.workspace_bytes)
for rep in range(6):
    rs.sort_device(x, y, k, ws=ws, plan_=p)
    torch.cuda.synchronize()
    d = ws[-256:].view(torch.int32).cpu().numpy().view("uint32").astype("int64")
    t0, tm, ts, te = d[10], d[11], d[8], d[9]
    print("us from first start: last work end %.2f, tail start %.2f, tail end %.2f" %
          ((tm - t0) / 100, (ts - t0) / 100, (te - t0) / 100), flush=True)
