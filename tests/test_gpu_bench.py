"""bench.py's output contract on the GPU box (the driver parses rank 0's JSON line): one small run
of each mode, checked for the keys and types the contract names. Sizes are small so the run
takes seconds; the numbers themselves are not checked."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def run_bench(*args):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_headline_contract():
    d = run_bench("--steps", "2", "--warmup", "1", "--keys", str(1 << 24), "--cpu-n", str(1 << 20), "--cpu-reps", "1",
                  "--cpu-rows", "18,24", "--configs-n", str((1 << 22) + 5), "--configs-reps", "5",
                  "--configs-cpu-n", str(1 << 20))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "vendor", "end_to_end"):
        assert k in d, k
    assert d["verified"] is True  # the timed output: sorted, same multiset as the input
    assert d["vendor"]["value"] > 0 and d["end_to_end"]["ms_per_sort"] > 0
    assert set(d["cpu_baseline"]["rows"]) == {"2^18", "2^24"}
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["dtype"] == "u32" and d["value"] > 0
    assert "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["cores"] == 1 and cb["value"] > 0
    # what ran, from the library itself
    assert d["config"]["lane_order_probe"] in (0, 1) and d["config"]["scatter_kernels"]
    assert rf["kernel"].startswith("rs_scatter")
    # the other BASELINE configurations, measured in the same run
    assert set(d["configs"]) == {"c2", "zipf", "c4"}
    for name, c in d["configs"].items():
        assert c["verified"] is True and c["plan_check"] == 0, name
        assert c["ms_per_sort"] > 0 and c["Mkeys_per_s"] > 0 and c["sorts"] == 5, name
        assert 0 < c["scatter"]["frac"] < 1 and c["scatter"]["bytes_per_key"] == (16 if c["pairs"] else 8), name
        assert c["scatter_kernels"], name
    assert d["configs"]["c4"]["pairs"] and d["configs"]["c2"]["k_bits"] == 4
    # BASELINE.md §3's CPU row beside every configuration: Baseline1 at the config's k
    # (C2: k = 4), the oracle's pairs port for C4 (Baseline1 carries no payload)
    for name, c in d["configs"].items():
        cb = c["cpu_baseline"]
        assert cb["cores"] == 1 and cb["value"] > 0 and f"k={c['k_bits']}" in cb["sample"], (name, cb)
        assert str(1 << 20) in cb["sample"]
    assert d["configs"]["c2"]["cpu_baseline"]["kind"] in ("reference", "port")
    assert d["configs"]["c4"]["cpu_baseline"]["kind"] == "port" and "pairs" in d["configs"]["c4"]["cpu_baseline"]["sample"]


def test_bench_group_chunks_reported():
    d = run_bench("--steps", "1", "--warmup", "1", "--keys", str(1 << 27), "--no-cpu", "--configs", "")
    assert d["config"]["group_chunk_passes"] in ([1, 3], [])  # [] on a device with other than 256 chunks
    d = run_bench("--steps", "1", "--warmup", "1", "--keys", str(1 << 27), "--no-cpu", "--no-group-chunks", "--configs", "")
    assert d["config"]["group_chunk_passes"] == []


def test_bench_primitives_and_dist_path():
    d = run_bench("--primitives", "--steps", "2", "--warmup", "1", "--keys", str(1 << 24), "--configs", "")
    for k in ("copy", "histogram", "scan", "scatter", "local_sort", "partition_8"):
        assert d["primitives"][k]["ms"] > 0, k
    for impl, extra in (("c", []), ("c", ["--dist-full"]), ("c", ["--dist-full", "--dist-overlap"]), ("torch", [])):
        d = run_bench("--dist-path", "--dist-impl", impl, "--steps", "1", "--warmup", "1", "--keys", str(1 << 24),
                      "--no-cpu", *extra)
        assert d["value"] > 0 and "range-partition" in d["config"]["parallelism"] and d["verified"] is True
        assert ("full protocol" in d["config"]["parallelism"]) == ("--dist-full" in extra)


def test_bench_pairs_zipf_verified():
    d = run_bench("--steps", "1", "--warmup", "1", "--keys", str(1 << 24), "--dist", "zipf", "--pairs", "--no-cpu",
                  "--configs", "")
    assert d["verified"] is True and d["config"]["pairs"] is True


def run_bench_env(env_extra, *args, timeout=300):
    import os
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=str(ROOT), env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-2000:])
    return json.loads(lines[0])


def check_multi_block(d, world):
    m = d["multi"]
    assert m["transport_world"] == world and m["halves"] in (1, 2) and m["exchange_rounds"] >= 0
    ph = m["phases_ms_per_step"]
    for k in ("plan", "partition", "exchange", "local_sort", "total"):
        assert ph[k] >= 0, k
    assert ph["total"] > 0 and ph["local_sort"] > 0
    assert len(m["phases_ms_per_rank"]) == world and len(m["keys_out_per_rank"]) == world
    ex = m["exchange"]
    assert len(ex["bytes_sent_per_rank"]) == world and len(ex["bytes_recv_per_rank"]) == world
    # every key leaves its rank or stays in its own range: sent + own = the rank's input bytes
    n = d["config"]["keys_per_gpu"]
    for r in range(world):
        assert ex["bytes_sent_per_rank"][r] + ex["own_range_bytes_per_rank"][r] == n * ex["bytes_per_key"]
    assert sum(ex["bytes_sent_per_rank"]) == sum(ex["bytes_recv_per_rank"])
    assert sum(m["keys_out_per_rank"]) == n * world
    ls = m["local_sort_scatter"]
    assert ls is not None and 0 < ls["frac"] < 1 and ls["avg_launch_ms"] > 0
    # the top-level roofline is the local sort's scatter kernel, never a partition instance
    sys.path.insert(0, str(ROOT))
    from bench import is_partition_kernel
    kernel = d["roofline"]["kernel"].split(" (")[0]
    assert kernel.startswith("rs_scatter") and not is_partition_kernel(kernel), kernel
    assert any(is_partition_kernel(k) for k in d["config"]["scatter_kernels"])
    if world > 1:
        assert m["partition_scatter"] is not None and m["partition_scatter"]["avg_launch_ms"] > 0
    # the component-measured prediction the first real N-GPU run is checked against
    # (profiles/r06_multi_model.json; world 1: the direct sort)
    assert m["predicted_ms_per_step"] is not None and m["predicted_ms_per_step"] > 0
    assert m["prediction"]["halves"] == m["halves"] and m["prediction"]["link_64GBs_ms"] >= m["predicted_ms_per_step"]


def test_bench_plain_gpus2_self_launches_rehearsal():
    """`python bench.py --gpus 2` started plainly (no torch.distributed.run, as the driver may):
    bench.py starts the two ranks itself; RSORT_BENCH_BACKEND=gloo lets both share the one card
    (the C protocol over a gloo host transport; RCCL refuses two ranks on one GPU)."""
    d = run_bench_env({"RSORT_BENCH_BACKEND": "gloo"}, "--gpus", "2", "--steps", "2", "--warmup", "1",
                      "--keys", str((1 << 22) + 333), "--cpu-n", str(1 << 18), "--cpu-reps", "1", "--cpu-rows", "")
    assert d["n_gpus"] == 2 and d["verified"] is True and d["value"] > 0
    assert "range-partition x2" in d["config"]["parallelism"] and "gloo" in d["config"]["parallelism"]
    assert d["multi"]["rccl_world"] is None  # (no RCCL communicator in the rehearsal)
    check_multi_block(d, 2)
    assert d["multi"]["exchange"]["link_GBs"]["links"] == 2
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1


def test_bench_gpus2_overlap_pairs_rehearsal():
    d = run_bench_env({"RSORT_BENCH_BACKEND": "gloo"}, "--gpus", "2", "--steps", "1", "--warmup", "1",
                      "--keys", str(1 << 21), "--dist", "zipf", "--pairs", "--dist-overlap", "--no-cpu")
    assert d["n_gpus"] == 2 and d["verified"] is True
    check_multi_block(d, 2)
    assert d["multi"]["halves"] == 2 and d["multi"]["exchange"]["bytes_per_key"] == 8
    assert ", overlap" in d["config"]["parallelism"]
    # --no-overlap: one half per rank (the default at N = 2 is the overlap, rsort.h)
    d = run_bench_env({"RSORT_BENCH_BACKEND": "gloo"}, "--gpus", "2", "--steps", "1", "--warmup", "1",
                      "--keys", str(1 << 21), "--no-overlap", "--no-cpu")
    assert d["verified"] is True and d["multi"]["halves"] == 1 and ", overlap" not in d["config"]["parallelism"]


def test_bench_one_rank_rccl_reports_phases():
    """One rank over RCCL, the whole protocol: rccl_world comes from ncclCommCount."""
    d = run_bench_env({}, "--dist-path", "--dist-full", "--steps", "1", "--warmup", "1", "--keys", str(1 << 22),
                      "--no-cpu")
    assert d["verified"] is True and d["multi"]["rccl_world"] == 1
    check_multi_block(d, 1)


def test_bench_one_rank_direct_phases():
    """One rank without RSORT_MULTI_FULL sorts directly: the phase record is all local sort."""
    d = run_bench_env({}, "--dist-path", "--steps", "2", "--warmup", "1", "--keys", str(1 << 22), "--no-cpu")
    m = d["multi"]
    assert d["verified"] is True and m["rccl_world"] == 1
    ph = m["phases_ms_per_step"]
    assert ph["local_sort"] >= 0.9 * ph["total"] and ph["exchange"] <= 0.1 * ph["total"], ph
    assert m["local_sort_scatter"]["launches_per_step"] == d["config"]["passes"]


def test_bench_plain_gpus4_rehearsal_ragged():
    """Four ranks on the one card (gloo host transport), an odd key count per rank and all-equal keys
    (one equal-keys bucket split across every rank): the line, the checks and the per-rank record."""
    d = run_bench_env({"RSORT_BENCH_BACKEND": "gloo"}, "--gpus", "4", "--steps", "1", "--warmup", "1",
                      "--keys", str((1 << 20) + 77), "--dist", "equal", "--no-cpu")
    assert d["n_gpus"] == 4 and d["verified"] is True
    check_multi_block(d, 4)
    # one key everywhere: the equal-keys bucket is cut across the ranks evenly
    outs = d["multi"]["keys_out_per_rank"]
    assert max(outs) - min(outs) <= 0.05 * sum(outs) / 4 + 64, outs


def test_bench_gpus2_stalled_rank_ends_with_an_error():
    """the first real N-GPU run must not hang or end without a word. One rehearsal rank
    stalls before its first collective (RSORT_BENCH_STALL_RANK, a test hook), as a dead peer would:
    `bench.py --gpus 2` must exit non-zero within its launch timeout with a message, and leave no
    process of the run behind (the ranks and the launcher are one process group, killed on expiry)."""
    import os
    import time
    import uuid
    psutil = pytest.importorskip("psutil")
    tag = uuid.uuid4().hex
    env = dict(os.environ, RSORT_BENCH_BACKEND="gloo", RSORT_BENCH_STALL_RANK="1", RSORT_BENCH_TAG=tag)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--keys", str(1 << 20), "--no-cpu", "--launch-timeout", "60"], capture_output=True, text=True,
                       timeout=200, cwd=str(ROOT), env=env)
    el = time.monotonic() - t0
    assert r.returncode != 0, r.stdout[-1000:]
    assert el < 60 + 20 + 30, el  # (limit + the kill's grace periods + interpreter start)
    assert "stalls" in r.stderr or "did not finish" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]  # no line from a failed run
    time.sleep(2)
    left = []
    for p in psutil.process_iter():
        try:
            if p.environ().get("RSORT_BENCH_TAG") == tag:
                left.append((p.pid, p.cmdline()[:4]))
        except (psutil.AccessDenied, psutil.NoSuchProcess, psutil.ZombieProcess):
            continue
    assert not left, left
