"""Turn a profiles/run_profiles.sh output directory into the committed summaries.

    python profiles/summarize.py gpurun_out/prof_r01 r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_pmc.json: per-kernel FETCH_SIZE / WRITE_SIZE per launch and the HBM bytes per
scatter launch, corrected as MI355X_MICROARCH.md prescribes for gfx950 and calibrated in-run:
  - FETCH_SIZE counts KiB; on gfx950 it reports half the bytes of a coalesced streaming read.
    Calibration in this run: rs_histogram reads exactly n*4 bytes (16-B loads) -> ratio 0.5.
  - WRITE_SIZE counts KiB; exact for 16-B-per-lane stores (MI355X_MICROARCH.md) and, as
    calibrated in this run, for dword stores: rs_gen_uniform writes exactly n*4 bytes -> 1.0.
bench.py reads hbm_bytes_per_launch from this file for roofline.traffic.
"""
from __future__ import annotations

import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

HERE = Path(__file__).resolve().parent


def _counters(path: Path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def _one(glob_dir: Path, pattern: str) -> Path:
    hits = sorted(glob_dir.rglob(pattern))
    if not hits:
        raise SystemExit(f"no {pattern} under {glob_dir}")
    return hits[0]


def main(src: str, tag: str, n: int = 1 << 30, k: int = 8):
    src = Path(src)
    stats = _one(src / "trace", "*kernel_stats.csv")
    shutil.copy(stats, HERE / f"{tag}_kernel_stats.csv")
    fetch = _counters(_one(src / "pmc_fetch", "*counter_collection.csv"))
    write = _counters(_one(src / "pmc_write", "*counter_collection.csv"))

    def per_launch(agg, counter, needle):
        vals = [v for (kn, c), vs in agg.items() if c == counter and needle in kn for v in vs]
        return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)

    hist_fetch, _ = per_launch(fetch, "FETCH_SIZE", "rs_histogram")
    gen_write, _ = per_launch(write, "WRITE_SIZE", "rs_gen_uniform")
    sc_fetch, nf = per_launch(fetch, "FETCH_SIZE", "rs_scatter")
    sc_write, nw = per_launch(write, "WRITE_SIZE", "rs_scatter")
    kib = 1024.0
    fetch_ratio = (hist_fetch * kib) / (4.0 * n) if hist_fetch else 0.5
    write_ratio = (gen_write * kib) / (4.0 * n) if gen_write else 1.0
    read_bytes = sc_fetch * kib / fetch_ratio
    write_bytes = sc_write * kib / write_ratio
    algo = 8.0 * n
    names = {kn for (kn, c) in list(fetch) + list(write) if "rs_scatter" in kn}
    kernel = "rs_scatter_lines" if any("rs_scatter_lines" in kn for kn in names) else "rs_scatter"
    rows = {}
    for (kn, c), vs in sorted(fetch.items()) + sorted(write.items()):
        rows.setdefault(kn, {})[c + "_KiB_per_launch"] = sum(vs) / len(vs)
        rows[kn]["launches_" + c] = len(vs)
    out = {
        "source": f"profiles/run_profiles.sh {tag} (rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, "
                  f"separate passes; bench.py --steps 2 --warmup 1 at n={n}, k={k})",
        "calibration": {"fetch_ratio_measured": round(fetch_ratio, 4),
                        "fetch_ratio_note": "rs_histogram reads exactly 4n bytes with 16-B loads; "
                                            "gfx950 FETCH_SIZE reports half (MI355X_MICROARCH.md HBM)",
                        "write_ratio_measured": round(write_ratio, 4),
                        "write_ratio_note": "rs_gen_uniform writes exactly 4n bytes with dword stores"},
        "configs": {
            f"n{n}_k{k}_uniform_keys_match:{kernel}": {
                "kernel": f"{kernel} (fused local sort + rank + scatter)",
                "kernel_symbols": sorted(names),
                "launches": {"fetch_pass": nf, "write_pass": nw},
                "read_bytes_per_launch": read_bytes,
                "write_bytes_per_launch": write_bytes,
                "hbm_bytes_per_launch": read_bytes + write_bytes,
                "algorithmic_bytes_per_launch": algo,
                "traffic_over_algorithmic": (read_bytes + write_bytes) / algo,
            }
        },
        "per_kernel_raw": rows,
    }
    (HERE / f"{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out["configs"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
