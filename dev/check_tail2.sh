# dev/check_tail2.sh -- next-digit / tail-scan tests (k = 3, 4), then the C2 bench and its kernel trace
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_groups.py -k "next_digit" -x -q --timeout 120 --timeout-method thread > gpurun_out/tail2_tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/tail2_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --keys 67108864 --k 4 > gpurun_out/tail2_c2.json 2> gpurun_out/tail2_c2.err
bash dev/kt.sh c2_new --keys 67108864 --k 4
