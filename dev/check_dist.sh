# dev/check_dist.sh -- one gpurun call: partition/multi GPU tests, then the multi-GPU sort path
# on one rank (RCCL) with a kernel trace.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "partition or multi or top" > gpurun_out/dist_tests.log 2>&1
timeout -k 10 180 python bench.py --no-cpu --dist-path > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
