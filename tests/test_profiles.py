"""The committed profile summaries are reproducible from profiles/ alone: every
config record of the newest *_pmc.json that names a per-launch CSV gives back its rocprof_avg_ns
(the timed working launches) and its rocprof_csv_avg_ns (the --stats file's AverageNs)."""
import csv
import json
from pathlib import Path

PROF = Path(__file__).resolve().parent.parent / "profiles"


def _records():
    for f in sorted(PROF.glob("r*_pmc.json")):
        for cfg, rec in json.loads(f.read_text())["configs"].items():
            if rec.get("rocprof_launches_csv"):
                yield f.name, cfg, rec


def test_profile_averages_recompute_from_committed_files():
    recs = list(_records())
    assert recs, "no profile record names its per-launch CSV"
    for fname, cfg, rec in recs:
        launches = PROF / Path(rec["rocprof_launches_csv"].split()[0]).name
        rows = list(csv.DictReader(open(launches)))
        timed = [int(r["duration_ns"]) for r in rows if r["timed"] == "1"]
        assert len(timed) == rec["rocprof_calls"], (fname, cfg)
        assert abs(sum(timed) / len(timed) - rec["rocprof_avg_ns"]) < 1.0, (fname, cfg)
        assert all(r["working"] == "1" for r in rows if r["timed"] == "1")
        stats = PROF / Path(rec["rocprof_csv_source"].split()[0]).name
        row = next(r for r in csv.DictReader(open(stats)) if r["Name"] == rec["rocprof_csv_symbol"])
        assert abs(float(row["AverageNs"]) - rec["rocprof_csv_avg_ns"]) < 1e-6, (fname, cfg)
        # the working symbol's launches in the trace are the --stats file's calls
        sym = rec["rocprof_csv_symbol"].split("(")[0].replace("void rsort::", "")
        assert sum(1 for r in rows if r["kernel"] == sym) == int(row["Calls"]), (fname, cfg)
