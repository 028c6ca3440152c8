# dev/check_dist.sh -- one gpurun call: partition/multi GPU tests, then the multi-GPU sort path
# on one rank (RCCL), keys and Zipf pairs.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or multi or top" > gpurun_out/dist_tests.log 2>&1
timeout -k 10 180 python -u bench.py --no-cpu --dist-path > gpurun_out/bd.out 2> gpurun_out/bd.err
timeout -k 10 180 python -u bench.py --no-cpu --dist-path --pairs --dist zipf > gpurun_out/bd4.out 2> gpurun_out/bd4.err
