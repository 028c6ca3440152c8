# dev/prof_zipf2.sh -- kernel traces of the zipf keys sort with and without segment chunks
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_zipf $R/gpurun_out/prof_zipfn
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_zipf -- python3 $R/bench.py --no-cpu --dist zipf --steps 2 --warmup 1 > $R/gpurun_out/prof_zipf.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_zipfn -- python3 $R/bench.py --no-cpu --dist zipf --steps 2 --warmup 1 --no-group-chunks > $R/gpurun_out/prof_zipfn.log 2>&1
