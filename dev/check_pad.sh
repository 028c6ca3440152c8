# dev/check_pad.sh -- one gpurun call: the whole GPU suite, then bench lines (C3 twice, Zipf, C4, C2)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pad_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/pad_c3.json 2> gpurun_out/pad_c3.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --dist zipf > gpurun_out/pad_zipf.json 2> gpurun_out/pad_zipf.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --pairs --dist zipf > gpurun_out/pad_c4.json 2> gpurun_out/pad_c4.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor --keys 67108864 --k 4 > gpurun_out/pad_c2.json 2> gpurun_out/pad_c2.err
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor > gpurun_out/pad_c3b.json 2> gpurun_out/pad_c3b.err
bash dev/kt.sh pad
