set -e
cd $GRAFT_REPO_ROOT
LAB_K4=1 timeout -k 10 120 ./dev/lines_lab 26 > gpurun_out/lab_k4b.log 2>&1
LAB_K4=1 timeout -k 10 120 ./dev/lines_lab 30 >> gpurun_out/lab_k4b.log 2>&1
