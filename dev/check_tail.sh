# dev/check_tail.sh -- one gpurun call: k = 3, 4 parity (tail-scanned tables) and the C2 bench with
# and without next-digit counts.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 > gpurun_out/tail_c2.json 2> gpurun_out/tail_c2.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 --no-group-chunks > gpurun_out/tail_c2off.json 2> gpurun_out/tail_c2off.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 3 > gpurun_out/tail_c2k3.json 2> gpurun_out/tail_c2k3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --k 4 > gpurun_out/tail_k4big.json 2> gpurun_out/tail_k4big.err
