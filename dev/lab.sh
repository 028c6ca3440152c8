#!/bin/bash
# dev/lab.sh -- the one lab runner for GPU sessions (gpurun): `bash dev/lab.sh <experiment> [args]`.
# Every GPU step runs under its own timeout; the script stops at the first crash / timeout (a plain
# test failure, pytest rc 1, does not stop it). Output goes to gpurun_out/<experiment>*.
#
#   round         pytest -m gpu (all) + the default bench line            (the round-end tiers)
#   pairs         the pairs tests + the C4 config, new 128-B kernel and 64-B kernel (RSORT_PAIRS64=1)
#   bench [args]  bench.py with extra args
#   prof [args]   rocprofv3 --kernel-trace --stats of bench.py with extra args (profiles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
exp=$1
shift
ok_or_stop() {  # pytest rc 0/1 continue, anything else (crash, timeout) stops the session
    local rc=$1
    echo "[lab] $2 rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
}
run_bench() {  # name, args...
    local name=$1
    shift
    timeout -k 10 300 python bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "[lab] bench $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    tail -c 2500 "gpurun_out/$name.json"
}
case "$exp" in
round)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 300 --timeout-method thread \
        > gpurun_out/round_tests.log 2>&1
    ok_or_stop $? pytest
    tail -n 3 gpurun_out/round_tests.log
    run_bench round_bench --steps 20 --warmup 5
    ;;
pairs)
    timeout -k 10 600 python -u -m pytest tests -m gpu -v -k "pairs or clustered or cut_plan or group" \
        --timeout 300 --timeout-method thread > gpurun_out/pairs_tests.log 2>&1
    ok_or_stop $? pytest
    grep -E "passed|failed|FAILED|Error" gpurun_out/pairs_tests.log | tail -n 12
    run_bench pairs_new --steps 5 --warmup 2 --keys 16777216 --no-cpu --no-vendor --no-e2e --configs c4,zipf "$@"
    RSORT_PAIRS64=1 run_bench pairs_64 --steps 5 --warmup 2 --keys 16777216 --no-cpu --no-vendor --no-e2e \
        --configs c4 "$@"
    ;;
bench)
    run_bench "bench_${LAB_TAG:-x}" "$@"
    ;;
prof)
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${LAB_TAG:-x} -o run -- \
        python bench.py "$@" > gpurun_out/prof_${LAB_TAG:-x}.log 2>&1
    echo "[lab] prof rc=$?"
    ;;
*)
    echo "unknown experiment: $exp"
    exit 2
    ;;
esac
