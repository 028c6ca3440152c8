# dev/check_cut3.sh -- full GPU test suite, then bench C3 / Zipf keys / C4 / all-equal
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cut_all.log 2>&1
for d in "" "--dist zipf" "--dist zipf --pairs" "--dist equal"; do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-vendor $d >> gpurun_out/cut_bench.jsonl 2>> gpurun_out/cut_bench.err
done
