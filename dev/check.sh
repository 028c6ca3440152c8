# dev/check.sh -- one gpurun call: GPU tests (assertion failures do not stop the script; faults,
# aborts and timeouts do), then the lines lab and the benches.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
timeout -k 10 120 ./dev/lines_lab 30 > gpurun_out/lab_lines9.log 2>&1
timeout -k 10 180 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf > gpurun_out/bench_zipf.json 2> gpurun_out/bench_zipf.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 180 python bench.py --no-cpu --keys 67108864 --k 4 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
