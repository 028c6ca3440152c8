"""dev/rk_lab2.py -- the multi-GPU step at world 1 phase by phase (GpuOps, shared workspace)."""
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
import radixsort as rs  # noqa: E402
import multi  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
n = 1 << 30
keys = rs.empty_u32(n, dev)
rs.gen_uniform(keys, 0x5EED)
ops = multi.GpuOps(dev)


def t(label, fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{label:40s} {e0.elapsed_time(e1):8.3f} ms", flush=True)
    return r


for rep in range(2):
    h = t("top_histogram", lambda: ops.top_histogram(keys, 12))
    pk, pv, starts = t("partition", lambda: ops.partition(keys, None, []))
    rk = torch.empty_like(pk)
    t("all_to_all_single", lambda: dist.all_to_all_single(rk, pk, [n], [n]))
    print("  rk ptr % 4096 =", rk.data_ptr() % 4096, " ws ptr % 4096 =", ops._ws.data_ptr() % 4096, flush=True)
    t("  local sort (shared ws)", lambda: ops.sort(rk, None, 8))
    t("  local sort again (shared ws)", lambda: ops.sort(rk, None, 8))
    t("  local sort (own ws)", lambda: rs.sort_device(rk, torch.empty_like(rk), 8))
    t("  sort of the original keys", lambda: rs.sort_device(keys, torch.empty_like(keys), 8))
    print("  pk == keys:", bool(torch.equal(pk, keys)), " rk == keys:", bool(torch.equal(rk, keys)), flush=True)
    x = rk.clone()
    t("  sort of a clone of rk", lambda: rs.sort_device(x, torch.empty_like(x), 8))
    ws = rs.workspace(rs.plan(n, 8).workspace_bytes, dev)
    o = torch.empty_like(x)
    rs.sort_device(x, o, 8, ws=ws)
    print("  group flags of rk's sort:", rs.group_flags(rs.plan(n, 8), ws), flush=True)
    rs.sort_device(keys, o, 8, ws=ws)
    print("  group flags of keys' sort:", rs.group_flags(rs.plan(n, 8), ws), flush=True)
    del pk, rk
dist.destroy_process_group()
