# dev/check_k4.sh -- full GPU suite, then C2 and 2^30 k=4 benches
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --no-cpu --keys 67108864 --k 4 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 180 python bench.py --no-cpu --k 4 > gpurun_out/bench_k4big.json 2> gpurun_out/bench_k4big.err
timeout -k 10 180 python bench.py --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
