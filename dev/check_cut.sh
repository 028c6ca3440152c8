# dev/check_cut.sh -- one gpurun call: group tests first (cut plans), then parity, bench C3 / Zipf / C4
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cut_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cut_tests2.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/cut_c3.json 2> gpurun_out/cut_c3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist zipf > gpurun_out/cut_zipf.json 2> gpurun_out/cut_zipf.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist zipf --pairs > gpurun_out/cut_c4.json 2> gpurun_out/cut_c4.err
