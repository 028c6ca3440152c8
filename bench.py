"""bench.py -- BASELINE.json's headline: Mkeys/s sorting 2^30 uniform uint32 (k=8) on MI355X,
plus the achieved HBM GB/s of the scatter pass against the roofline, and the reference's
sequential sort (Baseline1.cu:15-64, oracle/_ref) timed on this host's cores beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 1073741824] [--k 8]
                  [--dist uniform|zipf] [--pairs] [--rank match|split] [--no-cpu]

A step = one complete sort of the resident input (every pass: histogram, scan, fused local
sort + scatter), device-resident: inputs are generated in HBM before timing, the timed region
is K back-to-back sorts bracketed by barrier + synchronize. N>1 (launched by
torch.distributed.run, one process per GPU over RCCL): each rank holds n keys of one global
uniform stream (block-distributed), and a step is the full multi-GPU sort (histogram
all-reduce, partition, one all-to-all over xGMI, local sort) -> weak scaling.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
import radixsort as rs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys", "--n", dest="n", type=int, default=1 << 30, help="keys per GPU")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--pairs", action="store_true")
    ap.add_argument("--rank", choices=["match", "split"], default="match")
    ap.add_argument("--tiles-per-chunk", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=1 << 26, help="keys in the CPU-baseline sample")
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--vendor", action="store_true", help="also time rocPRIM's radix sort")
    ap.add_argument("--dist-path", action="store_true",
                    help="run the multi-GPU sort (partition, RCCL all-to-all, local sort) even on one "
                         "rank: its overhead against the single-GPU sort")
    ap.add_argument("--primitives", action="store_true",
                    help="time the pass primitives in isolation instead (SURVEY 8f row 3) and exit")
    ap.add_argument("--no-group-chunks", action="store_true",
                    help="every pass counts its own histogram (no digit-group chunks)")
    return ap.parse_args()


def traffic_for(config_key: str):
    """HBM bytes per scatter launch from the committed PMC profile (profiles/*pmc*.json), or None."""
    for f in sorted((ROOT / "profiles").glob("*pmc*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        rec = d.get("configs", {}).get(config_key)
        if rec and rec.get("hbm_bytes_per_launch"):
            return rec["hbm_bytes_per_launch"], f.name
    return None, None


def cpu_baseline(n, k, reps, dist):
    """Baseline1's sortByHost on this host, single thread: the reference's own code from
    oracle/_ref when it was built (kind "reference"), else the oracle port (kind "port")."""
    sys.path.insert(0, str(ROOT / "tests"))
    import _util  # test/bench infrastructure: the oracle loaders (never the product path)
    x = _util.uniform_keys(n) if dist == "uniform" else _util.zipf_keys(n)
    out = np.empty_like(x)
    ref = _util.ref_lib()
    if ref is not None:
        kind = "reference"
        fn = lambda: ref.ref_sort_by_host(_util._ptr(x), n, _util._ptr(out), k)  # noqa: E731
    else:
        kind = "port"
        fn = lambda: _util.oracle().oracle_sort_by_host(_util._ptr(x), n, _util._ptr(out), k)  # noqa: E731
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(n / med / 1e6, 2), "unit": "Mkeys/s", "cores": 1, "kind": kind,
            "sample": f"{n} {dist} u32 keys, k={k}, median of {reps} single-thread runs "
                      f"({med * 1e3:.0f} ms each) of Baseline1 sortByHost on {model or 'host CPU'} "
                      f"(host has {os.cpu_count()} logical CPUs)",
            "ms_per_sort": round(med * 1e3, 2)}


def primitives(a, dev):
    """SURVEY 8f row 3 -- the reference's primitive demos (Histogram.cu:17-33,
    PrefixSum-WorkEfficient.cu:81-216, MatrixTranspose.cu:90-243) as this library's pass
    primitives, each timed alone on n resident keys with HIP events (median of `steps`): the
    chunk histogram (its store IS the transpose), the table scan, the block-local sort, the
    fused rank + scatter, and a plain device copy as the HBM ceiling they are read against."""
    n, k = a.n, a.k
    keys = rs.empty_u32(n, dev)
    rs.gen_uniform(keys, 0x5EED)
    out = rs.empty_u32(n, dev)
    p = rs.plan(n, k, False, a.tiles_per_chunk)
    table = torch.empty(p.table_entries, dtype=torch.int32, device=dev)
    bsums = torch.empty(max(1, p.scan_blocks), dtype=torch.int32, device=dev)

    def timed(fn):
        for _ in range(max(1, a.warmup)):
            fn()
        ts = []
        for _ in range(a.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    rows = {}

    def row(name, ms, nbytes, what):
        rows[name] = {"ms": round(ms, 4), "bytes": int(nbytes), "GB/s": round(nbytes / (ms * 1e-3) / 1e9, 1),
                      "frac_of_peak": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "what": what}

    row("copy", timed(lambda: out.copy_(keys)), 8 * n, "torch device copy (read n + write n)")
    row("histogram", timed(lambda: rs.pass_histogram(p, keys, 0, table)), 4 * n,
        "rs_histogram: per-chunk digit counts, stored column-major (histogram + transpose)")
    rs.pass_histogram(p, keys, 0, table)
    row("scan", timed(lambda: rs.pass_scan(p, table, bsums)), 8 * p.table_entries,
        "rs_scan_reduce + rs_scan_down over the table (re-scans its own output: timing only)")
    rs.pass_histogram(p, keys, 0, table)
    rs.pass_scan(p, table, bsums)
    row("scatter", timed(lambda: rs.pass_scatter(p, keys, out, 0, table)), 8 * n,
        f"{rs.scatter_kernel_name(p)}: block-local rank + global scatter")
    row("local_sort", timed(lambda: rs.pass_local_sort(p, keys, out, 0)), 8 * n,
        "block-local stable sort of every tile (sortLocallyDataBlocks' result)")
    for nb in (1, 2, 8):
        # the multi-GPU step's stable partition into nb key ranges (uniform splitters)
        spl = [(i << 32) // nb for i in range(1, nb)]
        starts = torch.empty(nb + 1, dtype=torch.int32, device=dev)
        pws = rs.workspace(int(rs._lib().rsort_partition_workspace_size(n, nb, 0)), dev)
        row(f"partition_{nb}", timed(lambda: rs.partition_device(keys, out, spl, starts, ws=pws)), 12 * n,
            f"rsort_partition_device into {nb} key ranges (histogram 4n + scatter 8n bytes)")
        del pws
    print(json.dumps({"primitives": rows, "keys": n, "k_bits": k, "tile_keys": p.tile_keys,
                      "num_chunks": p.num_chunks, "steps": a.steps, "peak_GBs": HBM_PEAK_GBS}), flush=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    # RSORT_BENCH_BACKEND=gloo: rehearsal of the N>1 path with several ranks on fewer GPUs
    # (host-side exchange; timings meaningless). The driver's runs use RCCL, one rank per GPU.
    backend = os.environ.get("RSORT_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or a.dist_path
    if use_dist:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    rs.set_rank_algo(rs.RANK_SPLIT if a.rank == "split" else rs.RANK_MATCH)
    rs.set_group_chunks(not a.no_group_chunks)
    if a.primitives:
        if world == 1:
            primitives(a, dev)
        return

    n = a.n
    seed = 0x5EED + rank * n  # one global splitmix stream, block-distributed by index
    keys = rs.empty_u32(n, dev)
    if a.dist == "uniform":
        rs.gen_uniform(keys, seed)
    else:
        sys.path.insert(0, str(ROOT / "tests"))
        from _util import zipf_cdf_u32
        rs.gen_zipf(keys, rs.from_numpy_u32(zipf_cdf_u32(), dev), seed)
    vals = None
    if a.pairs:
        vals = rs.empty_u32(n, dev)
        rs.gen_iota(vals, rank * n)
    p = rs.plan(n, a.k, a.pairs, a.tiles_per_chunk)
    # the single-GPU sort's buffers (the multi-GPU step allocates its own)
    out = rs.empty_u32(n, dev) if not use_dist else None
    vout = rs.empty_u32(n, dev) if a.pairs and not use_dist else None
    ws = rs.workspace(p.workspace_bytes, dev) if not use_dist else None

    if use_dist:
        import multi
        ops = multi.GpuOps(dev)

        def step():
            return multi.dist_sort(keys, a.k, vals=vals, ops=ops)
    else:
        def step():
            rs.sort_device(keys, out, a.k, vals_in=vals, vals_out=vout, ws=ws, plan_=p)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    barrier()
    torch.cuda.synchronize()
    with rs.Profile() as prof:
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    barrier()
    groups = rs.group_flags(p, ws) if not use_dist else None
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())

    # per-kernel: the fused local-sort + scatter pass (the dominant kernel)
    sc = prof.times["scatter"]
    hi = prof.times["histogram"]
    scan = prof.times["scan"]
    bytes_per_key = 16 if a.pairs else 8
    scatter_ms = sc["ms"] / max(1, sc["launches"])
    keys_per_launch = sc["keys"] / max(1, sc["launches"])
    achieved = bytes_per_key * keys_per_launch / (scatter_ms * 1e-3) / 1e9
    kernel = rs.scatter_kernel_name(p) if not use_dist else "rs_scatter_lines (partition and sort passes)"
    cfg_key = f"n{n}_k{a.k}_{a.dist}_{'pairs' if a.pairs else 'keys'}_{a.rank}:{kernel}"
    traffic, traffic_src = traffic_for(cfg_key)

    vendor = None
    if a.vendor and world == 1:
        vo = rs.empty_u32(n, dev)
        vws = rs.workspace(int(rs._lib().rsort_vendor_workspace_size(n)), dev)
        rs.vendor_sort_device(keys, vo, ws=vws)
        torch.cuda.synchronize()
        tv = time.perf_counter()
        for _ in range(a.steps):
            rs.vendor_sort_device(keys, vo, ws=vws)
        torch.cuda.synchronize()
        tv = (time.perf_counter() - tv) / a.steps
        vendor = {"value": round(n / tv / 1e6, 1), "unit": "Mkeys/s", "ms_per_sort": round(tv * 1e3, 3),
                  "impl": "rocprim::radix_sort_keys"}
        del vo, vws

    if rank == 0:
        total_keys = n * world * a.steps
        line = {
            "metric": "Mkeys/s sorting 2^30 uniform uint32; scatter-pass achieved HBM GB/s",
            "value": round(total_keys / elapsed / 1e6, 1),
            "unit": "Mkeys/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 uniform u32, seed 0x5EED, generated in HBM)"
                    if a.dist == "uniform" else "synthetic (Zipf s=1.0 over 2^20 ranks, key=fmix32(rank))",
            "config": {"workload": f"sort {n} {'key+value pairs' if a.pairs else 'uint32 keys'} per GPU, "
                                   f"k={a.k} ({p.passes} passes), {a.dist}",
                       "keys_per_gpu": n, "k_bits": a.k, "passes": p.passes, "dist": a.dist,
                       "pairs": bool(a.pairs), "rank_algo": a.rank, "tile_keys": p.tile_keys,
                       "tiles_per_chunk": p.tiles_per_chunk, "num_chunks": p.num_chunks,
                       "group_chunk_passes": ([2 * i + 1 for i, f in enumerate(groups) if f]
                                              if groups is not None else None),
                       "parallelism": "single GPU" if not use_dist else f"range-partition x{world} (RCCL all-to-all)"},
            "roofline": {"bound": "hbm", "kernel": f"{kernel} (fused local sort + rank + scatter)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": int(bytes_per_key * keys_per_launch),
                         "avg_launch_ms": round(scatter_ms, 4)},
            "phases_ms_per_step": {"histogram": round(hi["ms"] / a.steps, 4), "scan": round(scan["ms"] / a.steps, 4),
                                   "scatter": round(sc["ms"] / a.steps, 4)},
        }
        if vendor:
            line["vendor"] = vendor
        if not use_dist and not a.no_cpu:
            line["cpu_baseline"] = cpu_baseline(min(a.cpu_n, n), a.k, a.cpu_reps, a.dist)
        print(json.dumps(line), flush=True)
    if use_dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
