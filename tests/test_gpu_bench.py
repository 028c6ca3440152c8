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
                  "--cpu-rows", "18,24", "--configs-n", str((1 << 22) + 5), "--configs-reps", "5")
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
