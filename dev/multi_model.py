"""dev/multi_model.py -- a component-measured prediction of the multi-GPU step (DESIGN §5 "Predicted
N-GPU step") and the CU-sharing cost of RSORT_MULTI_OVERLAP, on ONE GPU.

Per rank of an N-GPU weak-scaling step (2^30 uniform keys per GPU, k = 8) the phases are timed apart,
each uncontended, at N = 2, 4, 8:
  plan        the sample / splitter phase of the whole protocol at one rank (loopback transport,
              RSORT_MULTI_FULL, rsort_multi_last_stats), plus a modelled RCCL latency per all-gather
  partition   rsort_partition_device into the buckets rsort_multi_splitters_make gives for N ranks
              (N - 1 quantile keys of distinct keys, none hot: N buckets)
  local sort  the sort of what one rank receives: 2^30 keys inside one rank's key range (the arrival
              of N sources; uniform keys: their top log2 N bits are the rank's)
  exchange    modelled: (N - 1) / N of the rank's keys, n / N per peer, each pair of GPUs on its own
              xGMI link, all links in parallel, at an assumed per-direction link rate
Overlap: the lower half's sort (2^29 keys) alone and beside a stand-in for the upper half's exchange
(dev/overlap_lab.hip: `wgs` resident workgroups pacing a copy of the half's exchange bytes at the
links' aggregate rate), with the default plan and with fixed-chunk plans that leave CUs free.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC dev/overlap_lab.hip -o dev/liboverlap_lab.so
  python dev/multi_model.py [--out gpurun_out/multi_model.json] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
import radixsort as rs  # noqa: E402

N = 1 << 30
LINK_GBS = (64.0, 153.0)  # assumed per-direction xGMI rates: ~RCCL p2p practice / the nominal link figure
AG_LATENCY_MS = 0.05      # assumed per RCCL all-gather of a few KiB..MiB (three per step)


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), [round(t, 4) for t in ts]


def to_i32(x64):
    """u32 values held in an int64 tensor -> the same bits in int32 storage."""
    return torch.where(x64 >= (1 << 31), x64 - (1 << 32), x64).to(torch.int32)


def range_keys(n, world, r, dev, seed=0x5EED):
    """n uniform keys inside rank r's key range of `world` equal ranges (top log2(world) bits = r)."""
    lg = world.bit_length() - 1
    u = rs.empty_u32(n, dev)
    rs.gen_uniform(u, seed + 77 * r)
    x = (u.to(torch.int64) & 0xFFFFFFFF) >> lg
    x |= r << (32 - lg)
    del u
    return to_i32(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/multi_model.json")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--wgs", default="8,32")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    res = {"keys_per_gpu": N, "k_bits": 8, "reps": a.reps, "link_GBs_assumed": list(LINK_GBS),
           "allgather_latency_ms_assumed": AG_LATENCY_MS}

    keys = rs.empty_u32(N, dev)
    rs.gen_uniform(keys, 0x5EED)
    out = rs.empty_u32(N, dev)
    p = rs.plan(N, 8)
    ws = rs.workspace(p.workspace_bytes, dev)
    t1, ts = timed(lambda: rs.sort_device(keys, out, 8, ws=ws, plan_=p), a.reps)
    res["single_gpu_sort_ms"] = round(t1, 4)
    res["single_gpu_sort_runs"] = ts
    print(f"single-GPU sort {t1:.3f} ms", flush=True)

    # plan phase: the whole protocol at one rank (loopback transport), its phase record
    g = rs.LoopbackGroup(1)
    tr = g.transport(0)
    cap = rs.default_capacity(N)
    mout = rs.empty_u32(cap, dev)
    mws = rs.workspace(int(rs._lib().rsort_multi_workspace_size(N, cap, 8, 0, 1)), dev)
    stats = []
    with rs.multi_options(rs.MULTI_FULL):
        rs.multi_set_profiling(True)
        try:
            for i in range(a.reps + 1):
                rs.multi_sort_device(tr, keys, 8, capacity=cap, ws=mws, out=(mout, None))
                torch.cuda.synchronize()
                if i:
                    stats.append(rs.multi_last_stats())
        finally:
            rs.multi_set_profiling(False)
    g.close()
    del mout, mws
    ph = {k: round(float(np.median([s[k] for s in stats])), 4)
          for k in ("ms_plan", "ms_partition", "ms_exchange", "ms_local_sort", "ms_total")}
    res["world1_full_protocol_ms"] = ph
    print("world-1 full protocol", ph, flush=True)
    torch.cuda.empty_cache()

    def partition_ms(V):
        # the splitters rsort_u32_multi makes for V (virtual) ranks of distinct keys: no quantile key hot
        q = [(i << 32) // V for i in range(1, V)]
        splitters = rs.multi_splitters(V, q, hot=[0] * (V - 1)).splitters
        starts = torch.empty(len(splitters) + 2, dtype=torch.int32, device=dev)
        pws = rs.workspace(int(rs._lib().rsort_partition_workspace_size(N, len(splitters) + 1, 0)), dev)
        t, ts = timed(lambda: rs.partition_device(keys, out, splitters, starts, ws=pws), a.reps)
        del pws
        return t, ts, len(splitters) + 1

    res["worlds"] = {}
    for W in [int(x) for x in a.worlds.split(",")]:
        tp, tps, nbk = partition_ms(W)
        tpo, tpos, nbko = partition_ms(2 * W)  # the overlap's two halves per rank
        arr = range_keys(N, W, W // 2, dev)
        tl, tls = timed(lambda: rs.sort_device(arr, out, 8, ws=ws, plan_=p), a.reps)
        groups = rs.group_flags(p, ws)
        del arr
        torch.cuda.empty_cache()
        per_link = N // W * 4
        sent = (W - 1) * per_link
        row = {"buckets": nbk, "partition_ms": round(tp, 4), "partition_runs": tps,
               "overlap_buckets": nbko, "overlap_partition_ms": round(tpo, 4), "overlap_partition_runs": tpos,
               "local_sort_ms": round(tl, 4), "local_sort_runs": tls,
               "local_sort_group_modes": [("fixed", "groups", "cut")[f] for f in groups],
               "exchange_bytes_sent": sent, "bytes_per_link": per_link, "own_range_bytes": per_link,
               "predicted": {}}
        for L in LINK_GBS:
            tex = per_link / (L * 1e9) * 1e3
            step = ph["ms_plan"] + 3 * AG_LATENCY_MS + tp + tex + tl
            row["predicted"][f"link_{int(L)}GBs"] = {
                "exchange_ms": round(tex, 3), "ms_per_step": round(step, 3),
                "Gkeys_per_s": round(W * N / (step * 1e-3) / 1e9, 1),
                "weak_scaling_eff": round(t1 / step, 3)}
        res["worlds"][str(W)] = row
        print(f"W={W}: partition {tp:.3f} local sort {tl:.3f}", row["predicted"], flush=True)

    # ---- overlap: the lower half's sort beside a stand-in for the upper half's exchange
    lab = ctypes.CDLL(str(ROOT / "dev" / "liboverlap_lab.so"))
    lab.lab_hold.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                             ctypes.c_void_p]
    H = N // 2
    W = 8
    half = range_keys(H, 2 * W, W, dev)  # the lower half of rank 4's range at N = 8 (2N virtual ranks)
    hout = rs.empty_u32(H, dev)
    srcb = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    dstb = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    plans = {"default": rs.plan(H, 8)}
    tiles = (H + plans["default"].tile_keys - 1) // plans["default"].tile_keys
    for c in (224,):
        tpc = (tiles + c - 1) // c
        plans[f"fixed{(tiles + tpc - 1) // tpc}"] = rs.plan(H, 8, False, tpc)
    hws = rs.workspace(max(pp.workspace_bytes for pp in plans.values()), dev)
    ov = {"half_keys": H, "world": W, "plans": {}}
    for name, pp in plans.items():
        alone, _ = timed(lambda: rs.sort_device(half, hout, 8, ws=hws, plan_=pp), a.reps)
        prow = {"num_chunks": int(pp.num_chunks), "alone_ms": round(alone, 4), "contended": {}}
        for L in LINK_GBS:
            rate = (W - 1) * L  # GB/s over all links (read and written locally at this rate)
            hbytes = H // W * 4 * (W - 1)  # the upper half's exchange bytes out (and in)
            hbytes = min(hbytes, srcb.numel())
            for wg in [int(x) for x in a.wgs.split(",")]:
                ts_sort, ts_hold = [], []
                for rep in range(a.reps + 1):
                    torch.cuda.synchronize()
                    eh0, eh1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    with torch.cuda.stream(side):
                        eh0.record()
                        if lab.lab_hold(srcb.data_ptr(), dstb.data_ptr(), hbytes, wg, rate, side.cuda_stream):
                            raise RuntimeError("lab_hold failed")
                        eh1.record()
                    es0.record()
                    rs.sort_device(half, hout, 8, ws=hws, plan_=pp)
                    es1.record()
                    torch.cuda.synchronize()
                    if rep:
                        ts_sort.append(es0.elapsed_time(es1))
                        ts_hold.append(eh0.elapsed_time(eh1))
                prow["contended"][f"link_{int(L)}GBs_wgs{wg}"] = {
                    "sort_ms": round(float(np.median(ts_sort)), 4), "hold_ms": round(float(np.median(ts_hold)), 4),
                    "hold_bytes": int(hbytes), "hold_GBs": rate}
                print(name, L, wg, prow["contended"][f"link_{int(L)}GBs_wgs{wg}"], flush=True)
        # the hold alone (its duration without the sort)
        ov["plans"][name] = prow
    for L in LINK_GBS:
        th, _ = timed(lambda: lab.lab_hold(srcb.data_ptr(), dstb.data_ptr(), min(H // W * 4 * (W - 1), srcb.numel()),
                                           32, (W - 1) * L, torch.cuda.current_stream().cuda_stream), 3, warm=1)
        ov[f"hold_alone_ms_link_{int(L)}GBs"] = round(th, 4)
    res["overlap"] = ov
    # the sorted output of the last contended run is still a sort: check it
    fp_in = rs.fingerprint(half)[0]
    rs.sort_device(half, hout, 8, ws=hws, plan_=plans["default"])
    fp_out, desc = rs.fingerprint(hout)
    res["overlap_check"] = bool(fp_in == fp_out and desc == 0)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps({"done": a.out, "time": time.strftime("%H:%M:%S")}), flush=True)


if __name__ == "__main__":
    main()
