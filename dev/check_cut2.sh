# dev/check_cut2.sh -- group tests, then kernel traces of Zipf / all-equal / C3 sorts
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cut_tests.log 2>&1
bash dev/kt.sh zc --dist zipf
bash dev/kt.sh eq --dist equal
bash dev/kt.sh c3
