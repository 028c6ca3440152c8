# dev/check_part.sh -- one gpurun call: the whole GPU suite, primitives (partition rows), dist path
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --primitives --steps 5 > gpurun_out/prim_c3.json 2> gpurun_out/prim_c3.err
timeout -k 10 180 python -u bench.py --no-cpu --dist-path > gpurun_out/bd.out 2> gpurun_out/bd.err
timeout -k 10 180 python -u bench.py --no-cpu --dist-path --pairs --dist zipf > gpurun_out/bd4.out 2> gpurun_out/bd4.err
