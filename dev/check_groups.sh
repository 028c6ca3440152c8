# dev/check_groups.sh -- one gpurun call: segment-chunk tests, then benches with and without.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_groups.py -x -v --timeout 120 --timeout-method thread > gpurun_out/groups_tests.log 2>&1
timeout -k 10 180 python bench.py --no-cpu > gpurun_out/bench_groups.json 2> gpurun_out/bench_groups.err
timeout -k 10 180 python bench.py --no-cpu --no-group-chunks > gpurun_out/bench_nogroups.json 2> gpurun_out/bench_nogroups.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf > gpurun_out/bench_zipf.json 2> gpurun_out/bench_zipf.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs --no-group-chunks > gpurun_out/bench_c4n.json 2> gpurun_out/bench_c4n.err
