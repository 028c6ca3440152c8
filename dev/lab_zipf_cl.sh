# dev/lab_zipf_cl.sh -- uniform pass 0 and Zipf passes 1, 2 (fixed n/256 chunks ~ a cut plan) through
# the rank variants of the clustered kernels (timing only)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/lab_zcl.log
timeout -k 10 100 ./dev/lines_exp 30 "pad" >> gpurun_out/lab_zcl.log 2>&1
for p in 1 2; do
  LX_ZIPF=1 LX_PASS=$p timeout -k 10 100 ./dev/lines_exp 30 "pad" >> gpurun_out/lab_zcl.log 2>&1
done
