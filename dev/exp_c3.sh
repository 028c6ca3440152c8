# dev/exp_c3.sh V1 V2 ... -- kernel traces of the C3 bench per library variant dev/var_V.so
set -e
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  cp dev/var_$v.so cuda.radixsort_amd/librsort.so
  bash dev/kt.sh c3_$v
done
