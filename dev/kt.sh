# dev/kt.sh TAG [bench args] -- per-launch kernel trace of a short bench run (gpurun_out/kt_TAG)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_$TAG -- python3 $R/bench.py --no-cpu --no-e2e --no-vendor --steps 2 --warmup 1 "$@" > $R/gpurun_out/kt_$TAG.log 2>&1
