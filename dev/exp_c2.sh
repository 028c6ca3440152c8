# dev/exp_c2.sh V1 V2 ... -- kernel traces of the C2 bench (2^26 keys, k = 4) per library variant
set -e
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  cp dev/var_$v.so cuda.radixsort_amd/librsort.so
  bash dev/kt.sh c2_$v --keys 67108864 --k 4
done
