"""dev/rk_lab.py -- why is the first histogram over an RCCL all_to_all output slow?
World-1 RCCL group; times rs.pass_histogram (plain and in the full sort) on buffers written by
(a) rs_gen_uniform, (b) torch copy_, (c) all_to_all_single, each read twice."""
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
import radixsort as rs  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
n = 1 << 30
src = rs.empty_u32(n, dev)
rs.gen_uniform(src, 1)
p = rs.plan(n, 8)
table = torch.empty(p.table_entries, dtype=torch.int32, device=dev)


def t(label, fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{label:48s} {e0.elapsed_time(e1):8.3f} ms", flush=True)


for rep in range(2):
    dst = rs.empty_u32(n, dev)
    t("gen_uniform write", lambda: rs.gen_uniform(dst, 2))
    t("  hist #1", lambda: rs.pass_histogram(p, dst, 0, table))
    t("  hist #2", lambda: rs.pass_histogram(p, dst, 0, table))
    t("torch copy_ write", lambda: dst.copy_(src))
    t("  hist #1", lambda: rs.pass_histogram(p, dst, 0, table))
    t("all_to_all_single write", lambda: dist.all_to_all_single(dst, src))
    t("  hist #1", lambda: rs.pass_histogram(p, dst, 0, table))
    t("  hist #2", lambda: rs.pass_histogram(p, dst, 0, table))
    t("all_to_all_single write (splits)", lambda: dist.all_to_all_single(dst, src, [n], [n]))
    t("  hist #1", lambda: rs.pass_histogram(p, dst, 0, table))
    out = rs.empty_u32(n, dev)
    t("all_to_all_single write", lambda: dist.all_to_all_single(dst, src))
    t("  full sort (group chunks)", lambda: rs.sort_device(dst, out, 8))
    t("  full sort again", lambda: rs.sort_device(dst, out, 8))
    del dst, out
dist.destroy_process_group()
