set -e
cd $GRAFT_REPO_ROOT
LAB_ZIPF=1 timeout -k 10 120 ./dev/lines_lab 30 > gpurun_out/lab_lines23.log 2>&1
timeout -k 10 120 ./dev/lines_lab 30 >> gpurun_out/lab_lines23.log 2>&1
