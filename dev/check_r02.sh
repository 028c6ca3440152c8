# dev/check_r02.sh -- one gpurun call: GPU tests of the pass kernels, the line-kernel lab, then the
# bench lines of the BASELINE configs (C3 headline, Zipf keys, C4 Zipf pairs, C2 k=4).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_groups.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/chk_tests.log 2>&1
timeout -k 10 120 ./dev/lines_exp 30 > gpurun_out/chk_lab.log 2>&1
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/chk_c3.json 2> gpurun_out/chk_c3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --dist zipf > gpurun_out/chk_zipf.json 2> gpurun_out/chk_zipf.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --dist zipf --pairs > gpurun_out/chk_c4.json 2> gpurun_out/chk_c4.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 > gpurun_out/chk_c2.json 2> gpurun_out/chk_c2.err
