# dev/prof_all.sh -- one gpurun call: profiles/run_profiles.sh for C3, C4 and C2
set -e
cd $GRAFT_REPO_ROOT
bash profiles/run_profiles.sh r01
bash profiles/run_profiles.sh r01_c4 --dist zipf --pairs
bash profiles/run_profiles.sh r01_c2 --keys 67108864 --k 4
