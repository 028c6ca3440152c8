# dev/check_pairs.sh -- one gpurun call: pairs parity (dense 128-B-line pairs kernel), then bench
# lines of uniform pairs and C4, and a kernel trace of C4
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pairs or clustered" > gpurun_out/pairs_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --pairs > gpurun_out/pairs_u.json 2> gpurun_out/pairs_u.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --pairs --dist zipf > gpurun_out/pairs_c4.json 2> gpurun_out/pairs_c4.err
bash dev/kt.sh c4p --pairs --dist zipf
bash dev/kt.sh up --pairs
