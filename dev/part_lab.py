"""dev/part_lab.py -- the multi-GPU partition (rsort_partition_device) of 2^30 uniform keys into the
buckets of N ranks, timed per configuration (run under rocprofv3 --kernel-trace --stats to split it into
its histogram, scan and scatter kernels). Backs DESIGN §5 "Predicted N-GPU step".

  python dev/part_lab.py [--log2n 30] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
import radixsort as rs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = 1 << a.log2n
    dev = torch.device("cuda", 0)
    keys = rs.empty_u32(n, dev)
    rs.gen_uniform(keys, 0x5EED)
    out = rs.empty_u32(n, dev)
    cases = {}
    for W in (2, 4, 8):
        q = [(i << 32) // W for i in range(1, W)]
        cases[f"equal_buckets_w{W}"] = rs.multi_splitters(W, q).splitters
        cases[f"plain_w{W}"] = q
    cases["plain_w16"] = [(i << 32) // 16 for i in range(1, 16)]  # the overlap's 2N buckets at N = 8
    cases["equal_buckets_w16"] = rs.multi_splitters(16, cases["plain_w16"]).splitters  # every quantile hot: 31
    # unequal buckets: the chunks' output offsets inside a bucket are then no power-of-two stride apart
    cases["uneven_w2"] = [0x55555555]
    cases["uneven_w4"] = [0x30000000, 0x70000000, 0xB0000000]
    cases["one_bucket"] = []
    res = {}
    for name, spl in cases.items():
        nb = len(spl) + 1
        starts = torch.empty(nb + 1, dtype=torch.int32, device=dev)
        ws = rs.workspace(int(rs._lib().rsort_partition_workspace_size(n, nb, 0)), dev)
        for _ in range(2):
            rs.partition_device(keys, out, spl, starts, ws=ws)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rs.partition_device(keys, out, spl, starts, ws=ws)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[name] = {"buckets": nb, "ms": round(float(np.median(ts)), 4)}
        print(name, res[name], flush=True)
        del ws
    print(json.dumps(res))


if __name__ == "__main__":
    main()
