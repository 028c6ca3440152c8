# dev/check_prim.sh -- one gpurun call: new group tests, primitives microbench (C3, C2 shapes)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_groups.py -x -q --timeout 120 --timeout-method thread > gpurun_out/groups_tests.log 2>&1
timeout -k 10 180 python bench.py --primitives --steps 10 > gpurun_out/prim_c3.json 2> gpurun_out/prim_c3.err
timeout -k 10 180 python bench.py --primitives --steps 10 --keys 67108864 --k 4 > gpurun_out/prim_c2.json 2> gpurun_out/prim_c2.err
