# dev/prof_groups.sh -- one gpurun call: C4 with/without digit-group chunks (A/B on one box),
# then profiles/run_profiles.sh for C3 and C4.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs >> gpurun_out/ab_c4.jsonl 2>/dev/null
timeout -k 10 180 python bench.py --no-cpu --dist zipf --pairs --no-group-chunks >> gpurun_out/ab_c4.jsonl 2>/dev/null
done
bash profiles/run_profiles.sh r01
bash profiles/run_profiles.sh r01_c4 --dist zipf --pairs
