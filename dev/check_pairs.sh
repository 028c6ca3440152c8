# dev/check_pairs.sh -- pairs GPU tests, then the pairs benches (C4 and uniform pairs)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pairs or partition or multi or groups" > gpurun_out/pairs_tests.log 2>&1
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 180 python bench.py --no-cpu --pairs > gpurun_out/bench_upairs.json 2> gpurun_out/bench_upairs.err
timeout -k 10 180 python bench.py --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
