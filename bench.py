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
import contextlib
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


@contextlib.contextmanager
def stdout_to_stderr():
    """Library banners (gloo's peer count, RCCL's version block) print to fd 1 during setup; keep
    rank 0's stdout to the one JSON line the driver parses."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys", "--n", dest="n", type=int, default=1 << 30, help="keys per GPU")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--dist", choices=["uniform", "zipf", "equal", "hot", "zipf12"], default="uniform",
                    help="key distribution (equal: every key the same, the clustered extreme; hot: a quarter of "
                         "the keys one value at random positions, the rest uniform; zipf12: Zipf s=1.2)")
    ap.add_argument("--pairs", action="store_true")
    ap.add_argument("--rank", choices=["match", "split"], default="match")
    ap.add_argument("--tiles-per-chunk", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=1 << 26, help="keys in the CPU-baseline headline sample")
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--cpu-rows", default="20,30",
                    help="log2 sizes of extra Baseline1 rows (C1 = 2^20 and the GPU size), '' for none")
    ap.add_argument("--no-vendor", action="store_true", help="skip the rocPRIM radix sort column")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the reference-style host->host time (H2D + sort + D2H, Parallel7.cu:646-661)")
    ap.add_argument("--dist-impl", choices=["c", "torch"], default="c",
                    help="multi-GPU step: rsort_u32_multi over RCCL (c) or multi.py over torch.distributed")
    ap.add_argument("--dist-path", action="store_true",
                    help="run the multi-GPU sort (partition, RCCL all-to-all, local sort) even on one "
                         "rank: its overhead against the single-GPU sort")
    ap.add_argument("--dist-full", action="store_true",
                    help="multi-GPU step (c): the whole protocol also at one rank (RSORT_MULTI_FULL: sample, "
                         "partition, self exchange); by default one rank sorts directly")
    ap.add_argument("--dist-overlap", action="store_true",
                    help="multi-GPU step (c): RSORT_MULTI_OVERLAP at any world (sort each rank's lower half while "
                         "the upper half is exchanged); by default the library runs it for 2 <= N <= 4 only")
    ap.add_argument("--no-overlap", action="store_true",
                    help="multi-GPU step (c): RSORT_MULTI_NO_OVERLAP (one half per rank at every world)")
    ap.add_argument("--primitives", action="store_true",
                    help="time the pass primitives in isolation instead (SURVEY 8f row 3) and exit")
    ap.add_argument("--no-group-chunks", action="store_true",
                    help="every pass counts its own histogram (no digit-group chunks)")
    ap.add_argument("--configs", default="c2,zipf,c4",
                    help="BASELINE configurations measured after the headline in the same process, "
                         "reported in the line's `configs` block ('' for none; N=1 only): " + ", ".join(CONFIGS))
    ap.add_argument("--configs-n", type=int, default=0, help="override every config's key count (tests)")
    ap.add_argument("--configs-reps", type=int, default=7, help="timed sorts per config (median)")
    ap.add_argument("--configs-cpu-n", type=int, default=1 << 26,
                    help="keys of each config's CPU-baseline row (a prefix of its input; 0: none)")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="--gpus N without a launcher: seconds before the N ranks are killed and this command "
                         "exits non-zero (0: 300 s + 60 s per 2^30 keys over all ranks)")
    return ap.parse_args()


# BASELINE.json's other single-GPU configurations (configs[1], configs[3]) and the Zipf keys between
# them, measured in the same process after the headline (configs[2]) so the driver's run observes them
CONFIGS = {
    "c2": {"n": 1 << 26, "k": 4, "dist": "uniform", "pairs": False,
           "what": "C2 (BASELINE configs[1]): 2^26 uniform u32 keys, k=4"},
    "zipf": {"n": 1 << 30, "k": 8, "dist": "zipf", "pairs": False,
             "what": "2^30 Zipf(s=1) u32 keys, k=8 (C4's keys without the payload)"},
    "c4": {"n": 1 << 30, "k": 8, "dist": "zipf", "pairs": True,
           "what": "C4 (BASELINE configs[3]): 2^30 Zipf(s=1) u32 keys + u32 payloads (the input index), k=8"},
}


def profile_record(config_key: str):
    """The newest committed profile record of this configuration (profiles/*pmc*.json, newest
    round last): HBM bytes per scatter launch from the PMC passes and the rocprofv3 --stats
    average duration of the same kernel; (record, file name) or (None, None)."""
    best = (None, None)
    for f in sorted((ROOT / "profiles").glob("*pmc*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        rec = d.get("configs", {}).get(config_key)
        if rec and rec.get("hbm_bytes_per_launch"):
            best = (rec, f.name)
    return best


def _pin_one_core():
    """Pin this process to one CPU it may run on (os.sched_setaffinity, no re-exec); returns the
    previous set so the caller can restore it."""
    try:
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {min(old)})
        return old
    except (AttributeError, OSError):
        return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "host CPU"


def config_cpu_row(c, host_keys, host_vals, reps):
    """BASELINE.md §3's CPU row beside a GPU configuration: the reference's Baseline1 sortByHost
    (oracle/_ref, kind "reference") on a prefix of the config's own keys at its k -- or, for pairs
    (Baseline1 has no payload), the oracle's pairs port of the same loop (kind "port") -- ONE thread
    pinned to one core, median of `reps` runs."""
    sys.path.insert(0, str(ROOT / "tests"))
    import _util  # test/bench infrastructure (never the product path)
    k = c["k"]
    x = np.ascontiguousarray(host_keys)
    ko = np.empty_like(x)
    if host_vals is not None:
        v = np.ascontiguousarray(host_vals)
        vo = np.empty_like(v)
        kind, what = "port", "the oracle's pairs restatement of Baseline1 (Baseline1.cu:15-64 carrying a payload)"

        def run():
            _util.oracle().oracle_sort_pairs_by_host(_util._ptr(x), _util._ptr(v), x.size, _util._ptr(ko),
                                                     _util._ptr(vo), k)
    else:
        ref = _util.ref_lib()
        kind = "reference" if ref is not None else "port"
        what = "Baseline1 sortByHost" + (" (the reference's own code, oracle/_ref)" if ref is not None else
                                         " (the oracle's restatement)")

        def run():
            if ref is not None:
                ref.ref_sort_by_host(_util._ptr(x), x.size, _util._ptr(ko), k)
            else:
                _util.oracle().oracle_sort_by_host(_util._ptr(x), x.size, _util._ptr(ko), k)
    old = _pin_one_core()
    try:
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)
    med = float(np.median(ts))
    return {"value": round(x.size / med / 1e6, 2), "unit": "Mkeys/s", "cores": 1, "kind": kind,
            "sample": f"{x.size} {c['dist']} u32 {'key+value pairs' if host_vals is not None else 'keys'} "
                      f"(a prefix of this config's input), k={k}, median of {reps} runs of {what}, one thread "
                      f"pinned to one core of {_cpu_model()}",
            "ms_per_sort": round(med * 1e3, 2)}


def cpu_baseline(host_keys, n, k, reps, dist, rows):
    """Baseline1's sortByHost on this host, ONE thread pinned to one core: the reference's own code
    from oracle/_ref when it was built (kind "reference"), else the oracle port (kind "port").
    The headline value is the n-key sample (a prefix of the bench's own input, copied from HBM);
    `rows` adds more sizes (C1 = 2^20 and the GPU size), one run each above 2^26 keys."""
    sys.path.insert(0, str(ROOT / "tests"))
    import _util  # test/bench infrastructure: the oracle loaders (never the product path)
    ref = _util.ref_lib()
    kind = "reference" if ref is not None else "port"

    def run(x, out):
        if ref is not None:
            ref.ref_sort_by_host(_util._ptr(x), x.size, _util._ptr(out), k)
        else:
            _util.oracle().oracle_sort_by_host(_util._ptr(x), x.size, _util._ptr(out), k)

    old = _pin_one_core()
    try:
        def timed(m, nreps):
            x = np.ascontiguousarray(host_keys[:m])
            out = np.empty_like(x)
            ts = []
            for _ in range(nreps):
                t0 = time.perf_counter()
                run(x, out)
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts))

        med = timed(n, reps)
        extra = {}
        for lg in rows:
            m = 1 << lg
            if m > host_keys.size:
                continue
            t = timed(m, reps if m <= (1 << 26) else 1)
            extra[f"2^{lg}"] = {"keys": m, "Mkeys_per_s": round(m / t / 1e6, 2), "ms_per_sort": round(t * 1e3, 2),
                                "runs": reps if m <= (1 << 26) else 1}
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)
    return {"value": round(n / med / 1e6, 2), "unit": "Mkeys/s", "cores": 1, "kind": kind,
            "sample": f"{n} {dist} u32 keys (a prefix of the bench input), k={k}, median of {reps} runs "
                      f"({med * 1e3:.0f} ms each) of Baseline1 sortByHost, one thread pinned to one core of "
                      f"{_cpu_model()} (host has {os.cpu_count()} logical CPUs)",
            "ms_per_sort": round(med * 1e3, 2), "rows": extra}


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


def gen_keys(n, dist, seed, dev):
    keys = rs.empty_u32(n, dev)
    if dist == "uniform":
        rs.gen_uniform(keys, seed)
    elif dist == "equal":
        keys.fill_(0x1234567)
    elif dist == "hot":
        rs.gen_uniform(keys, seed)
        sel = rs.empty_u32(n, dev)
        rs.gen_uniform(sel, seed ^ 0x5A5A5A5A5A)
        keys[(sel & 3) == 0] = 0xC0FFEE
        del sel
    else:
        sys.path.insert(0, str(ROOT / "tests"))
        from _util import zipf_cdf_u32  # the workload's CDF table (data, not the oracle)
        cdf = zipf_cdf_u32(s=1.2) if dist == "zipf12" else zipf_cdf_u32()
        rs.gen_zipf(keys, rs.from_numpy_u32(cdf, dev), seed)
    return keys


def run_config(name, c, dev, reps, n_override=0, cpu_n=0, cpu_reps=3):
    """One BASELINE configuration, device-resident like the headline: after >= 0.25 s of warm-up
    sorts, ms per sort = the median of `reps` back-to-back sorts, each between two HIP events on the
    library's stream (torch's current stream); the scatter kernel's average launch time from HIP
    events around every scatter launch of 3 more sorts (rsort_profile_*); the output checked on the
    device (sorted, the input's multiset fingerprint)."""
    n = n_override or c["n"]
    keys = gen_keys(n, c["dist"], 0x5EED, dev)
    vals = None
    if c["pairs"]:
        vals = rs.empty_u32(n, dev)
        rs.gen_iota(vals, 0)
    fp_in = rs.fingerprint(keys, vals)[0]
    p = rs.plan(n, c["k"], c["pairs"])
    ws = rs.workspace(p.workspace_bytes, dev)
    out = rs.empty_u32(n, dev)
    vout = rs.empty_u32(n, dev) if c["pairs"] else None

    def step():
        rs.sort_device(keys, out, c["k"], vals_in=vals, vals_out=vout, ws=ws, plan_=p)

    rs.scatter_kernels_used(reset=True)
    # warm-up by time, not count: a config runs after host-side work (the end-to-end copy, the CPU
    # rows) that leaves the GPU idle and its clocks down, and two 1-ms sorts (C2) do not bring them
    # back (the same C2 library: 1.058 ms/sort in this block, 0.98-0.99 in runs without that idle
    # time); >= 0.25 s of sorts first, at least 2
    t0 = time.perf_counter()
    for i in range(400):
        step()
        if i >= 1 and i % 4 == 3:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= 0.25:
                break
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    med = ts[len(ts) // 2]
    with rs.Profile() as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    fp_out, desc = rs.fingerprint(out, vout)
    sc = prof.times["scatter"]
    launch_ms = sc["ms"] / max(1, sc["launches"])
    bpk = 16 if c["pairs"] else 8
    algo = bpk * sc["keys"] / max(1, sc["launches"])
    achieved = algo / (launch_ms * 1e-3) / 1e9
    groups = rs.group_flags(p, ws)
    res = {"what": c["what"], "keys": n, "k_bits": c["k"], "dist": c["dist"], "pairs": c["pairs"],
           "ms_per_sort": round(med, 3), "ms_per_sort_min_max": [round(ts[0], 3), round(ts[-1], 3)], "sorts": reps,
           "Mkeys_per_s": round(n / (med * 1e-3) / 1e6, 1),
           "scatter": {"avg_launch_ms": round(launch_ms, 4), "bytes_per_key": bpk,
                       "achieved_GBs": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                       "launches_per_sort": sc["launches"] // 3},
           "phases_ms_per_sort": {ph: round(prof.times[ph]["ms"] / 3, 4) for ph in ("histogram", "scan", "scatter")},
           "group_chunk_modes": [("fixed", "groups", "cut")[f] for f in groups] if p.k_bits == 8 else None,
           "scatter_kernels": rs.scatter_kernels_used(reset=True),
           "plan_check": rs.plan_check(p, ws),
           "verified": bool(fp_out == fp_in and desc == 0)}
    if cpu_n > 0:
        m = min(cpu_n, n)
        res["cpu_baseline"] = config_cpu_row(c, rs.to_numpy_u32(keys[:m]),
                                             rs.to_numpy_u32(vals[:m]) if vals is not None else None, cpu_reps)
    del keys, vals, out, vout, ws
    torch.cuda.empty_cache()
    return res


def visible_gpus() -> int:
    """GPUs this process may use, without touching HIP: HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES when set, else the render nodes (/dev/dri/renderD*) of the machine."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip()])
    return len(list(Path("/dev/dri").glob("renderD*")))


def launch_timeout(a) -> float:
    """Seconds the N ranks of a self-launched run may take: --launch-timeout, else 300 s (a fresh box's
    first `import torch`, RCCL setup) + 60 s per 2^30 keys over all ranks (the CPU baseline and the
    configs run at N = 1 only)."""
    return a.launch_timeout if a.launch_timeout > 0 else 300.0 + 60.0 * a.n * a.gpus / (1 << 30)


def self_launch(a) -> int:
    """`--gpus N` (N > 1) started plainly, without torch.distributed.run: start the N ranks as ONE
    child `python -m torch.distributed.run` (127.0.0.1, a free port) running this same command line,
    in a process group of its own, and return its exit code. The run is bounded: past launch_timeout
    the whole group is killed (SIGTERM, then SIGKILL) and this exits 124 with a message, so a stalled
    rank (a peer that died, a collective that never completes) ends the command instead of hanging it.
    This process never initialises HIP (it counts GPUs from the environment / device nodes) and never
    re-execs; the children inherit stdout, so rank 0's JSON line is this command's output."""
    import socket
    visible = visible_gpus()
    if os.environ.get("RSORT_BENCH_BACKEND", "") != "gloo" and visible < a.gpus:
        print(f"bench.py: --gpus {a.gpus} but {visible} GPU(s) visible (RSORT_BENCH_BACKEND=gloo rehearses "
              f"N ranks on fewer GPUs)", file=sys.stderr)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # (RCCL over dmabuf IPC on these hosts)
    limit = launch_timeout(a)
    env["RSORT_BENCH_TIMEOUT"] = str(int(limit))  # (the ranks bound their own collectives below it)
    return run_group(cmd, env, limit, f"the {a.gpus} ranks")


def run_group(cmd, env, limit, what, grace=10.0) -> int:
    """Run cmd in a process group of its own and return its exit code; past `limit` seconds kill the
    whole group (SIGTERM, then SIGKILL after `grace`) and return 124 with a message on stderr."""
    import signal
    import subprocess
    sys.stdout.flush()
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait(timeout=limit)
    except subprocess.TimeoutExpired:
        print(f"bench.py: {what} did not finish within {limit:.0f} s (a stalled or dead rank); "
              f"killing process group {proc.pid}", file=sys.stderr, flush=True)
        for sig in (signal.SIGTERM, signal.SIGKILL):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        # (the group may outlive its leader: make sure nothing of it is left)
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        return 124
    except BaseException:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        raise


def _template_args(name):
    return [x.strip() for x in name.split("<", 1)[1].rstrip(">").split(",")] if "<" in name else []


def is_partition_kernel(name):
    """A multi-GPU partition's scatter instance (splitter digits: DMODE = kDigitSplit = 1, template
    argument 5 of rs_scatter / rs_scatter_lines; rs_scatter_pairs never partitions)."""
    args = _template_args(name)
    return name.split("<")[0] in ("rs_scatter", "rs_scatter_lines") and len(args) > 5 and args[5] == "1"


MULTI_MODEL = "r06_multi_model.json"  # profiles/: the one-GPU component measurements (dev/multi_model.py)


def predict_multi_step(model, world, halves, link_gbs):
    """The multi-GPU step's time per rank predicted from components measured on ONE GPU (DESIGN §5
    "Predicted N-GPU step"): plan (+ an assumed latency per RCCL all-gather) + partition into the buckets
    of `world` ranks (2 x world with the overlap's halves) + the exchange, n / world keys per peer over each
    pair's own xGMI link at `link_gbs`, all links in parallel + the local sort of the 2^30-key arrival.
    With two halves, each half's exchange moves half the bytes; the lower half's sort runs during the upper
    half's exchange at the measured CU-shared rate (its time alone / its time beside a stand-in for the
    exchange's resident kernels), the rest after it; then the upper half's sort. world 1: the direct sort."""
    if world <= 1:
        return model["single_gpu_sort_ms"]
    w = model["worlds"].get(str(world))
    if w is None:
        return None
    base = model["world1_full_protocol_ms"]["ms_plan"] + 3 * model["allgather_latency_ms_assumed"]
    ex = w["bytes_per_link"] / (link_gbs * 1e9) * 1e3
    if halves == 1:
        return base + w["partition_ms"] + ex + w["local_sort_ms"]
    ov = model["overlap"]["plans"]["default"]
    half_alone = ov["alone_ms"]
    shared = ov["contended"].get(f"link_{int(link_gbs)}GBs_wgs8", {}).get("sort_ms", 2 * half_alone)
    rate = half_alone / shared
    e_half = ex / 2
    done = min(half_alone, rate * e_half)
    return base + w["overlap_partition_ms"] + 2 * e_half + (half_alone - done) + half_alone


def multi_prediction(world, halves):
    """multi.predicted_ms_per_step of the N > 1 line (at the nominal 153-GB/s link rate) and its
    alternative at the ~64 GB/s RCCL point-to-point rates reach in practice; None without the model."""
    try:
        model = json.loads((ROOT / "profiles" / MULTI_MODEL).read_text())
    except (OSError, ValueError):
        return None, None
    main = predict_multi_step(model, world, halves, 153.0)
    alt = predict_multi_step(model, world, halves, 64.0)
    return (round(main, 3) if main is not None else None,
            {"link_64GBs_ms": round(alt, 3) if alt is not None else None, "link_153GBs_ms": round(main, 3)
             if main is not None else None, "halves": halves,
             "source": f"profiles/{MULTI_MODEL} (dev/multi_model.py, one GPU) + bench.predict_multi_step"})


def multi_summary(per_rank, world, rank_of_stats, transport, sc, pt, steps):
    """The N-GPU block of the line: per-phase ms (mean over the profiled steps per rank, max over
    ranks), the exchange's bytes per rank and per peer link, and the local sort's and the partition's
    own scatter rooflines. per_rank: every rank's list of rsort_multi_stats dicts (one per step)."""
    ph = ("ms_plan", "ms_partition", "ms_exchange", "ms_local_sort", "ms_total")
    means = [{k: float(np.mean([st[k] for st in steps])) for k in ph} for steps in per_rank]
    last = [steps[-1] for steps in per_rank]
    bpk = last[0]["bytes_per_key"]
    sent = [sum(x["send_keys"][p] for p in range(world) if p != r) * bpk for r, x in enumerate(last)]
    recv = [sum(x["recv_keys"][p] for p in range(world) if p != r) * bpk for r, x in enumerate(last)]
    own = [x["send_keys"][r] * bpk for r, x in enumerate(last)]
    links = []  # (src, dst, bytes, GB/s over the source rank's exchange phase)
    for r, x in enumerate(last):
        for p in range(world):
            if p != r and x["send_keys"][p]:
                b = x["send_keys"][p] * bpk
                links.append((r, p, b, b / (means[r]["ms_exchange"] * 1e-3) / 1e9 if means[r]["ms_exchange"] else None))
    rates = [l[3] for l in links if l[3]]
    ex_ms = max(m["ms_exchange"] for m in means)

    def roof(t, what):
        if not t["launches"]:
            return None
        ms = t["ms"] / t["launches"]
        algo = 8 * t["keys"] / t["launches"] * (2 if last[0]["bytes_per_key"] == 8 else 1)
        return {"what": what, "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": int(algo),
                "achieved": round(algo / (ms * 1e-3) / 1e9, 1), "frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "launches_per_step": t["launches"] // max(1, steps)}

    pred, pred_detail = multi_prediction(world, int(last[0]["halves"]))
    return {
        "transport": transport,
        "predicted_ms_per_step": pred,
        "prediction": pred_detail,
        "rccl_world": rank_of_stats.get("rccl_world"),
        "transport_world": int(last[0]["world"]),
        "halves": int(last[0]["halves"]), "exchange_rounds": int(last[0]["rounds"]),
        "phases_ms_per_step": {k[3:]: round(max(m[k] for m in means), 4) for k in ph},
        "phases_ms_per_rank": [{k[3:]: round(m[k], 4) for k in ph} for m in means],
        "keys_out_per_rank": [int(x["n_out"]) for x in last],
        "exchange": {"bytes_per_key": int(bpk), "bytes_sent_per_rank": sent, "bytes_recv_per_rank": recv,
                     "own_range_bytes_per_rank": own,
                     "GBs_out_per_rank": [round(b / (m["ms_exchange"] * 1e-3) / 1e9, 2) if m["ms_exchange"] else None
                                          for b, m in zip(sent, means)],
                     "link_GBs": {"min": round(min(rates), 2), "mean": round(float(np.mean(rates)), 2),
                                  "max": round(max(rates), 2), "links": len(rates)} if rates else None,
                     "busiest_link_bytes": max((l[2] for l in links), default=0),
                     "ms": round(ex_ms, 4)},
        "local_sort_scatter": roof(sc, "the local sort's scatter passes (rank 0, 8 B/key keys, 16 B/key pairs)"),
        "partition_scatter": roof(pt, "the key-range partition's scatter (rank 0, splitter digits)"),
    }


def main():
    a = parse()
    # --gpus N without a launcher: start the N ranks here (before anything touches the GPU)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; running {world} ranks", file=sys.stderr)
    # RSORT_BENCH_BACKEND=gloo: rehearsal of the N>1 path with several ranks on fewer GPUs (the C
    # protocol over a gloo host transport; timings meaningless). The driver's runs use RCCL.
    rehearsal = os.environ.get("RSORT_BENCH_BACKEND", "") == "gloo"
    if rehearsal:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or a.dist_path
    dist = None
    if use_dist:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # control plane (barriers, the time max, the RCCL id) on gloo; the keys move over RCCL:
        # rsort_u32_multi's own communicator (c) or torch's nccl process group (torch). Every wait is
        # bounded: gloo's collectives and RCCL's steps (rsort_set_comm_timeout) time out below the
        # launcher's limit, so a stalled peer ends the run with an error instead of a hang
        import datetime
        limit = float(os.environ.get("RSORT_BENCH_TIMEOUT", "600"))
        to = datetime.timedelta(seconds=max(30.0, limit - 60.0))
        rs.set_comm_timeout(int(max(30.0, limit - 90.0) * 1000))
        with stdout_to_stderr():
            if a.dist_impl == "torch" and not rehearsal:
                dist.init_process_group("nccl", device_id=dev, timeout=to)
            else:
                dist.init_process_group("gloo", timeout=to)
    # TEST HOOK (tests/test_gpu_bench.py): this rank stalls before its first collective, as a dead peer
    # would; its peers then wait in that collective until the timeouts above or the launcher end them
    if os.environ.get("RSORT_BENCH_STALL_RANK", "") == str(rank) and world > 1:
        print(f"bench.py: rank {rank} stalls (RSORT_BENCH_STALL_RANK)", file=sys.stderr, flush=True)
        time.sleep(10 ** 6)
    rs.set_rank_algo(rs.RANK_SPLIT if a.rank == "split" else rs.RANK_MATCH)
    rs.set_group_chunks(not a.no_group_chunks)
    if a.primitives:
        if world == 1:
            primitives(a, dev)
        return

    n = a.n
    seed = 0x5EED + rank * n  # one global splitmix stream, block-distributed by index
    keys = gen_keys(n, a.dist, seed, dev)
    vals = None
    if a.pairs:
        vals = rs.empty_u32(n, dev)
        rs.gen_iota(vals, rank * n)
    fp_in = rs.fingerprint(keys, vals)[0]
    p = rs.plan(n, a.k, a.pairs, a.tiles_per_chunk)

    comm = None
    host_tr = None
    transport = None
    rccl_world = None
    if use_dist and a.dist_impl == "c":
        rs.set_multi_options((rs.MULTI_FULL if a.dist_full else 0) | (rs.MULTI_OVERLAP if a.dist_overlap else 0) |
                             (rs.MULTI_NO_OVERLAP if a.no_overlap and not a.dist_overlap else 0))
        if rehearsal:
            import multi
            host_tr = multi.host_transport()
            comm = host_tr.transport
            transport = f"gloo host transport (rehearsal: {world} ranks on {torch.cuda.device_count()} GPU(s))"
        else:
            uid = [rs.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            with stdout_to_stderr():
                comm = rs.RcclComm(world, rank, uid[0])
            transport = "RCCL (rsort_u32_multi: grouped ncclSend/ncclRecv over xGMI)"
        cap = rs.default_capacity(n)
        out = rs.empty_u32(cap, dev)
        vout = rs.empty_u32(cap, dev) if a.pairs else None
        ws = rs.workspace(int(rs._lib().rsort_multi_workspace_size(n, cap, a.k, int(a.pairs), world)), dev)
        res = {}

        def step():
            res["out"] = rs.multi_sort_device(comm, keys, a.k, vals=vals, capacity=cap, ws=ws, out=(out, vout))
    elif use_dist:
        import multi
        ops = multi.GpuOps(dev)
        res = {}
        transport = "torch.distributed all_to_all (multi.py)" + (" over gloo (rehearsal)" if rehearsal else " over RCCL")

        def step():
            res["out"] = multi.dist_sort(keys, a.k, vals=vals, ops=ops)
    else:
        out = rs.empty_u32(n, dev)
        vout = rs.empty_u32(n, dev) if a.pairs else None
        ws = rs.workspace(p.workspace_bytes, dev)

        def step():
            rs.sort_device(keys, out, a.k, vals_in=vals, vals_out=vout, ws=ws, plan_=p)

    rs.scatter_kernels_used(reset=True)
    with stdout_to_stderr():  # torch's nccl group connects on its first collective
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    # per-phase HIP events in a second, separate set of steps: the event records between the
    # phases cost ~10 us each (~85 us per C3 sort, rocprofv3 kernel trace), so `value` is timed
    # without them and the roofline's per-launch kernel times come from these steps; the multi-GPU
    # sort also records its own phase boundaries there (rsort_multi_set_profiling)
    multi_stats = []
    prof_c = use_dist and a.dist_impl == "c"
    barrier()
    if prof_c:
        rs.multi_set_profiling(True)
    try:
        with rs.Profile() as prof:
            for _ in range(a.steps):
                step()
                if prof_c:
                    multi_stats.append(rs.multi_last_stats())
            torch.cuda.synchronize()
    finally:
        if prof_c:
            rs.multi_set_profiling(False)
    barrier()
    if prof_c and comm is not None and not rehearsal:
        rccl_world = int(multi_stats[-1]["world"])  # rsort_u32_multi takes it from ncclCommCount

    # the timed output, checked on the device: sorted, same (key, value) multiset as the input
    # (summed over ranks for the multi-GPU step: each rank's slice is sorted, and the slices are
    # in order across ranks -- rank r's last key <= rank r + 1's first)
    if use_dist:
        ok, ov, _ = res["out"]
        fp_out, desc = rs.fingerprint(ok, ov)

        def s64(x):  # u64 fingerprint as an int64 tensor element
            return x - (1 << 64) if x >= (1 << 63) else x
        first = int(ok[0].item()) & 0xFFFFFFFF if ok.numel() else -1
        last = int(ok[-1].item()) & 0xFFFFFFFF if ok.numel() else -1
        mine = torch.tensor([s64(fp_in), s64(fp_out), desc, ok.numel(), first, last], dtype=torch.int64)
        parts = [torch.zeros(6, dtype=torch.int64) for _ in range(world)]
        if world > 1:
            dist.all_gather(parts, mine)
        else:
            parts = [mine]
        parts = [[int(v) for v in x] for x in parts]
        fin = sum(x[0] for x in parts) & 0xFFFFFFFFFFFFFFFF
        fout = sum(x[1] for x in parts) & 0xFFFFFFFFFFFFFFFF
        nonempty = [x for x in parts if x[3] > 0]
        ordered = all(nonempty[i][5] <= nonempty[i + 1][4] for i in range(len(nonempty) - 1))
        verified = (fin == fout and sum(x[2] for x in parts) == 0 and ordered
                    and sum(x[3] for x in parts) == n * world)
        per_rank_stats = [multi_stats]
        if world > 1 and prof_c:
            per_rank_stats = [None] * world
            dist.all_gather_object(per_rank_stats, multi_stats)
    else:
        fp_out, desc = rs.fingerprint(out, vout)
        verified = fp_out == fp_in and desc == 0
    groups = rs.group_flags(p, ws) if not use_dist else None
    kernels_used = rs.scatter_kernels_used(reset=True)  # what the dispatch launched in these steps
    probe = rs.lane_order_probe()

    # per-kernel: the fused local-sort + scatter pass (the dominant kernel); in the multi-GPU step
    # the partition's scatter is recorded apart (phase "partition") and the sample sort not at all
    sc = prof.times["scatter"]
    hi = prof.times["histogram"]
    scan = prof.times["scan"]
    bytes_per_key = 16 if a.pairs else 8
    scatter_ms = sc["ms"] / max(1, sc["launches"])
    keys_per_launch = sc["keys"] / max(1, sc["launches"])
    algo_bytes = bytes_per_key * keys_per_launch
    achieved = algo_bytes / (scatter_ms * 1e-3) / 1e9 if scatter_ms > 0 else 0.0
    # the pass's working kernel: the plain variant where a clustered-input twin (the same name ending
    # in ", 1>" instead of ", 0>") was launched beside it; never a partition instance
    sort_kernels = [k for k in kernels_used if not is_partition_kernel(k)]
    plain = [k for k in sort_kernels if not (k.endswith(", 1>") and k[:-2] + "0>" in sort_kernels)]
    kernel = plain[-1] if plain else rs.scatter_kernel_name(p)
    cfg_key = f"n{n}_k{a.k}_{a.dist}_{'pairs' if a.pairs else 'keys'}_{a.rank}:{kernel.split('<')[0]}"
    prec, prec_src = profile_record(cfg_key) if not use_dist else (None, None)

    vendor = None
    if not a.no_vendor and not use_dist and not a.pairs:
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
                  "impl": "rocprim::radix_sort_keys (what sortByThrust resolves to on ROCm, Parallel7.cu:69-73)",
                  "ours_over_vendor": round((n / (elapsed / a.steps)) / (n / tv), 2)}
        del vo, vws

    host_keys = None
    e2e = None
    if rank == 0 and ((not a.no_cpu) or (not a.no_e2e and not use_dist)):
        host_keys = rs.to_numpy_u32(keys)  # (rank 0's own input keys in the multi-GPU step)
    if host_keys is not None and not a.no_e2e and not a.pairs and not use_dist:
        # the reference's timing of sort(..., SORT_BY_DEVICE): device malloc + H2D + sort + D2H of
        # pageable host buffers (Parallel7.cu:646-661), through rsort_u32_ex; PCIe-bound, not `value`
        hout = np.empty_like(host_keys)
        rs.sortByDevice(host_keys, n, hout, a.k)  # first call sizes the library's cached workspace
        te = time.perf_counter()
        rs.sortByDevice(host_keys, n, hout, a.k)
        te = time.perf_counter() - te
        e2e = {"ms_per_sort": round(te * 1e3, 2), "Mkeys_per_s": round(n / te / 1e6, 1),
               "what": "host->host sortByDevice (H2D + sort + D2H, pageable buffers, Parallel7.cu:646-661)"}
        del hout

    configs = None
    if not use_dist and a.configs.strip():
        # the other BASELINE configurations, driver-observed: same process, after the headline
        del keys, vals, out, vout, ws
        torch.cuda.empty_cache()
        configs = {}
        for name in [x.strip() for x in a.configs.split(",") if x.strip()]:
            configs[name] = run_config(name, CONFIGS[name], dev, a.configs_reps, a.configs_n,
                                       0 if (a.no_cpu or rank != 0) else a.configs_cpu_n, a.cpu_reps)

    cpu = None
    if rank == 0 and host_keys is not None and not a.no_cpu:
        rows = [int(x) for x in a.cpu_rows.split(",") if x.strip()]
        cpu = cpu_baseline(host_keys, min(a.cpu_n, n), a.k, a.cpu_reps, a.dist, rows)

    if rank == 0:
        total_keys = n * world * a.steps
        roof = {"bound": "hbm", "kernel": f"{kernel} (fused local sort + rank + scatter"
                                          f"{'; the local sort after the exchange' if use_dist else ''})",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": prec["hbm_bytes_per_launch"] if prec else None,
                "traffic_source": prec_src,
                "algorithmic_bytes_per_launch": int(algo_bytes),
                "avg_launch_ms": round(scatter_ms, 4),
                "avg_launch_source": "HIP events around every scatter launch of a second set of `steps` steps "
                                     "(value is timed without events)"}
        if prec and prec.get("rocprof_avg_ns"):
            rp = prec["rocprof_avg_ns"] * 1e-6
            roof["avg_launch_ms_rocprof"] = round(rp, 4)
            roof["frac_rocprof"] = round(algo_bytes / (rp * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            roof["rocprof_source"] = prec.get("rocprof_source")
            if prec.get("rocprof_csv_avg_ns"):
                rc = prec["rocprof_csv_avg_ns"] * 1e-6
                roof["avg_launch_ms_rocprof_csv"] = round(rc, 4)
                roof["frac_rocprof_csv"] = round(algo_bytes / (rc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                roof["rocprof_csv_source"] = prec.get("rocprof_csv_source")
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
            "data": {"uniform": "synthetic (splitmix64 uniform u32, seed 0x5EED, generated in HBM)",
                     "zipf": "synthetic (Zipf s=1.0 over 2^20 ranks, key=fmix32(rank))",
                     "zipf12": "synthetic (Zipf s=1.2 over 2^20 ranks, key=fmix32(rank))",
                     "hot": "synthetic (uniform u32, a quarter of the positions set to 0x00C0FFEE)",
                     "equal": "synthetic (every key 0x01234567)"}[a.dist],
            "config": {"workload": f"sort {n} {'key+value pairs' if a.pairs else 'uint32 keys'} per GPU, "
                                   f"k={a.k} ({p.passes} passes), {a.dist}"
                                   + (f"; {world} ranks, key-range partition + one exchange + local sort"
                                      if use_dist else ""),
                       "keys_per_gpu": n, "k_bits": a.k, "passes": p.passes, "dist": a.dist,
                       "pairs": bool(a.pairs), "rank_algo": a.rank, "tile_keys": p.tile_keys,
                       "tiles_per_chunk": p.tiles_per_chunk, "num_chunks": p.num_chunks,
                       "group_chunk_passes": ([2 * i + 1 for i, f in enumerate(groups) if f]
                                              if groups is not None else None),
                       # per odd pass: its digit groups, equal chunks cutting unbalanced groups, or
                       # fixed chunks with a counted histogram (rsort_group_flags)
                       "group_chunk_modes": ([("fixed", "groups", "cut")[f] for f in groups]
                                             if groups is not None else None),
                       # the scatter instantiations the library's dispatch launched in the timed
                       # steps (rsort_scatter_kernels_used), and the ranking the probe allowed
                       "scatter_kernels": kernels_used,
                       "lane_order_probe": probe,
                       "ranking": ("lane-ordered returning LDS adds (kRankAtomic)" if probe == 1 and a.rank == "match"
                                   else "wave64 ballot peer match (kRankCount)" if a.rank == "match"
                                   else "k 1-bit splits (kRankSplit)"),
                       "parallelism": "single GPU" if not use_dist else
                       f"range-partition x{world} ({transport}"
                       f"{', overlap' if a.dist_impl == 'c' and prof_c and multi_stats and multi_stats[-1]['halves'] == 2 else ''}"
                       f"{', full protocol' if a.dist_full and a.dist_impl == 'c' else ''})"},
            "verified": bool(verified),
            "roofline": roof,
            "phases_ms_per_step": {"histogram": round(hi["ms"] / a.steps, 4), "scan": round(scan["ms"] / a.steps, 4),
                                   "scatter": round(sc["ms"] / a.steps, 4)},
        }
        if use_dist and prof_c:
            line["multi"] = multi_summary(per_rank_stats, world, {"rccl_world": rccl_world}, transport, sc,
                                          prof.times["partition"], a.steps)
        if configs:
            line["configs"] = configs
        if vendor:
            line["vendor"] = vendor
        if e2e:
            line["end_to_end"] = e2e
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if host_tr is not None:
        barrier()
        host_tr.close()
    if comm is not None and host_tr is None:
        comm.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
