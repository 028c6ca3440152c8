set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/chk9_tests.log 2>&1
timeout -k 10 120 ./dev/lines_exp 30 > gpurun_out/chk9_lab.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 > gpurun_out/chk9_c2.json 2> gpurun_out/chk9_c2.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 --no-group-chunks > gpurun_out/chk9_c2off.json 2> gpurun_out/chk9_c2off.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --k 4 > gpurun_out/chk9_k4big.json 2> gpurun_out/chk9_k4big.err
