# dev/check_jagg.sh -- one gpurun call: group/parity/fullsize tests, bench C3 (x2), all-equal keys, Zipf keys, kernel trace of all-equal
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ja_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/ja_c3.json 2> gpurun_out/ja_c3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist equal > gpurun_out/ja_eq.json 2> gpurun_out/ja_eq.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist zipf > gpurun_out/ja_zipf.json 2> gpurun_out/ja_zipf.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/ja_c3b.json 2> gpurun_out/ja_c3b.err
bash dev/kt.sh eq --dist equal
