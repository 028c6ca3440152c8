set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./dev/lines_lab 30 > gpurun_out/lab_lines11.log 2>&1
