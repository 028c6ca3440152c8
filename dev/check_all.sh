# dev/check_all.sh -- one gpurun call: the whole GPU test suite (assertion failures do not stop
# the script; faults, aborts and timeouts do), then the bench lines of every config.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
timeout -k 10 180 python bench.py --no-cpu --no-e2e --dist zipf > gpurun_out/bench_zipf.json 2> gpurun_out/bench_zipf.err
timeout -k 10 180 python bench.py --no-cpu --no-e2e --dist zipf --pairs > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 180 python bench.py --no-cpu --no-e2e --pairs > gpurun_out/bench_upairs.json 2> gpurun_out/bench_upairs.err
timeout -k 10 180 python bench.py --no-cpu --no-e2e --keys 67108864 --k 4 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 180 python bench.py --no-cpu --no-e2e --dist-path > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
