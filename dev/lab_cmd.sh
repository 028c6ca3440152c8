set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./dev/lines_lab_stamps 30 "k8 1024x16 lines" > gpurun_out/lab_lines8.log 2>&1
