# Kernel traces of 2^30 Zipf-key sorts with the cut plans' pieces from per-chunk rows (RSORT_PIECE_ROWS=1,
# the default) and counted from the keys (=0), RSORT_LAB=1: per kernel name, calls and mean us.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
for v in 1 0; do
    rm -rf "$R/gpurun_out/prows$v"
    (cd /tmp && RSORT_LAB=1 RSORT_PIECE_ROWS=$v TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$R/gpurun_out/prows$v" -- python3 "$R/bench.py" --keys 1073741824 --dist ${DIST:-zipf} ${PAIRS:-} --steps 4 \
        --warmup 1 --no-cpu --no-vendor --no-e2e --configs "" > "$R/gpurun_out/prows$v.log" 2>&1) || exit 1
done
for v in 1 0; do
    f=$(find "$R/gpurun_out/prows$v" -name "*kernel_trace.csv" | head -1)
    echo "== RSORT_PIECE_ROWS=$v"
    python3 - "$f" <<'PY'
import csv, sys, collections
t = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    t[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(t.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) > 100:
        print("  %-64s %4d %9.1f us mean, max %9.1f" % (k[:64], len(v), sum(v) / len(v), max(v)))
PY
done
