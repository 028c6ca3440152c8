# dev/prof_r02.sh -- one gpurun call: profiles/run_profiles.sh for C3, Zipf keys, C4 and C2, and a
# kernel trace of the multi-GPU step on one rank (round-2 profiles)
set -e
cd $GRAFT_REPO_ROOT
bash profiles/run_profiles.sh r02
bash profiles/run_profiles.sh r02_zipf --dist zipf
bash profiles/run_profiles.sh r02_c4 --dist zipf --pairs
bash profiles/run_profiles.sh r02_c2 --keys 67108864 --k 4
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_r02_dist
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02_dist -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --dist-path --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r02_dist.log 2>&1
