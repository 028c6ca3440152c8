# dev/check_defer.sh -- pairs tests, then pairs benches (uniform, Zipf) with kernel traces
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "pair" -x -q --timeout 300 --timeout-method thread > gpurun_out/defer_tests.log 2>&1
bash dev/kt.sh pu --pairs
bash dev/kt.sh pz --pairs --dist zipf
