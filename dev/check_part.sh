# dev/check_part.sh -- partition / multi-GPU tests, then the one-rank multi-GPU step and its kernel trace
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "multi or partition or dist" -x -q --timeout 300 --timeout-method thread > gpurun_out/part_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-vendor --dist-path > gpurun_out/part_dist.json 2> gpurun_out/part_dist.err
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/kt_part
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kt_part -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-vendor --dist-path --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/kt_part.log 2>&1
