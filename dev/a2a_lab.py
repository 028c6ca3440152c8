# Backs DESIGN §5 step 6: this RCCL leaves the second half of a >= 2 GiB message unwritten (1 GiB arrives whole).
"""dev/a2a_lab.py -- does all_to_all_single (RCCL, world 1) copy large int32 messages?"""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29535")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
for m in [1 << 20, 1 << 28, (1 << 29) - 1, 1 << 29, (1 << 29) + 1, 3 << 28, (1 << 30) - 5, 1 << 30]:
    src = torch.randint(-2**31, 2**31 - 1, (m,), dtype=torch.int32, device=dev)
    for variant in ("splits", "plain"):
        dst = torch.full((m,), 7, dtype=torch.int32, device=dev)
        if variant == "splits":
            dist.all_to_all_single(dst, src, [m], [m])
        else:
            dist.all_to_all_single(dst, src)
        torch.cuda.synchronize()
        ok = bool(torch.equal(dst, src))
        nbad = int((dst != src).sum().item())
        first_bad = int(torch.nonzero(dst != src)[0].item()) if nbad else -1
        print(f"m={m:11d} bytes={4*m:11d} {variant:6s} equal={ok} bad={nbad} first_bad={first_bad}", flush=True)
    del src, dst
    torch.cuda.empty_cache()
dist.destroy_process_group()
