# dev/bench3.sh -- one gpurun call: GPU tests, then repeated headline benches and the skewed configs.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do timeout -k 10 180 python bench.py --no-cpu --steps 10 >> gpurun_out/bench_rep.jsonl 2>/dev/null; done
timeout -k 10 180 python bench.py --no-cpu --dist zipf > gpurun_out/bench_zipf.json 2> gpurun_out/bench_zipf.err
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
