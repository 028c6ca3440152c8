#!/usr/bin/env bash
# profiles/run_profiles.sh -- the profiling recipe behind profiles/*.{csv,json,txt}.
# Run on the MI355X box from the repo root (gpurun). Every GPU step has its own time limit and
# the steps are chained with &&, so the first failure ends the script.
#   1. rocprofv3 --kernel-trace --stats of the default bench (per-kernel average durations)
#   2. two separate PMC passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass on gfx950)
#      of a 2-step bench, for the HBM traffic of the scatter kernel
# Output: gpurun_out/prof_${TAG}/ ; profiles/summarize.py turns it into the committed summaries.
set -euo pipefail
TAG="${1:-r01}"
shift || true
ARGS="$*"   # extra bench.py arguments, e.g. "--dist zipf --pairs" or "--keys 67108864 --k 4"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/prof_${TAG}"
rm -rf "$OUT"   # rocprofv3 writes per-process subdirectories: start clean
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-vendor --no-e2e --configs "" $ARGS > "$OUT/bench_trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-vendor --no-e2e --configs "" $ARGS > "$OUT/bench_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-vendor --no-e2e --configs "" $ARGS > "$OUT/bench_write.log" 2>&1
echo "profiles written to $OUT"
