"""dev/tail_stamps.py -- with a library variant built with -DRS_TAIL_STAMPS (dev/build_variant.sh), time
the phases of the last pass's tail scan at C2 (s_memrealtime, 100 MHz) from the workspace's tail area."""
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
for rep in range(5):
    rs.sort_device(x, y, k, ws=ws, plan_=p)
    torch.cuda.synchronize()
    tail = ws[-256:].view(torch.int32).cpu().numpy().view("uint32")
    st = [int(tail[8 + 2 * i]) | (int(tail[9 + 2 * i]) << 32) for i in range(4)]
    print("tail phases (us): sum sweep + wave totals %.2f, scan sweep + stores %.2f, zeroing %.2f" %
          ((st[1] - st[0]) / 100, (st[2] - st[1]) / 100, (st[3] - st[2]) / 100), flush=True)
