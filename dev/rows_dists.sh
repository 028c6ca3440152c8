# Cut plans' piece rows on other skewed inputs (RSORT_PIECE_ROWS=1 default vs 0, RSORT_LAB=1): ms per sort
# of bench.py --dist hot / zipf12 / zipf at 2^28, keys and pairs, alternating twice (gpurun_out/rows_dists.log)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
: > gpurun_out/rows_dists.log
for rep in 1 2; do
    for args in "--dist hot" "--dist zipf12" "--dist zipf --keys 268435456" "--dist hot --pairs"; do
        for v in 1 0; do
            RSORT_LAB=1 RSORT_PIECE_ROWS=$v timeout -k 10 200 python bench.py $args --steps 10 --warmup 3 --no-cpu \
                --no-vendor --no-e2e --configs "" > gpurun_out/rows_dists.json 2> gpurun_out/rows_dists.err || exit 1
            python3 - "$v" "$args" <<'PY' >> gpurun_out/rows_dists.log
import json, sys
d = json.loads(open("gpurun_out/rows_dists.json").read().strip().splitlines()[-1])
print("rows=%s %-28s %8.3f ms/sort  hist %.3f  verified %s" % (sys.argv[1], sys.argv[2], d["ms_per_step"],
      d["phases_ms_per_step"]["histogram"], d["verified"]))
PY
        done
    done
done
cat gpurun_out/rows_dists.log
