# dev/lab_rank.sh -- rank-variant lab (dev/lines_exp): uniform pass 0/1, Zipf passes 0..3
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/lab_rank.log
timeout -k 10 100 ./dev/lines_exp 30 >> gpurun_out/lab_rank.log 2>&1
LX_PASS=1 timeout -k 10 100 ./dev/lines_exp 30 >> gpurun_out/lab_rank.log 2>&1
for p in 0 1 2 3; do LX_ZIPF=1 LX_PASS=$p timeout -k 10 100 ./dev/lines_exp 30 >> gpurun_out/lab_rank.log 2>&1; done

