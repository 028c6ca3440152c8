# dev/check_cl.sh -- one gpurun call: group/parity tests (clustered kernels), then the bench lines
# of C3 (uniform keys), Zipf keys, C4 (Zipf pairs) and uniform pairs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cl_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/cl_c3.json 2> gpurun_out/cl_c3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist zipf > gpurun_out/cl_zipf.json 2> gpurun_out/cl_zipf.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --dist zipf --pairs > gpurun_out/cl_c4.json 2> gpurun_out/cl_c4.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --pairs > gpurun_out/cl_upairs.json 2> gpurun_out/cl_upairs.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/cl_c3b.json 2> gpurun_out/cl_c3b.err
