# dev/prof_all.sh -- one gpurun call: profiles/run_profiles.sh for C3, C4 and C2, and a kernel
# trace of the multi-GPU step on one rank
set -e
cd $GRAFT_REPO_ROOT
bash profiles/run_profiles.sh r01
bash profiles/run_profiles.sh r01_c4 --dist zipf --pairs
bash profiles/run_profiles.sh r01_c2 --keys 67108864 --k 4
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_dist
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dist -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --dist-path --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_dist.log 2>&1
