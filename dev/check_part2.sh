# dev/check_part2.sh -- partition/multi GPU tests, then the partition primitives
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or multi or top or groups" > gpurun_out/dist_tests.log 2>&1
timeout -k 10 180 python bench.py --primitives --steps 5 > gpurun_out/prim_c3.json 2> gpurun_out/prim_c3.err
