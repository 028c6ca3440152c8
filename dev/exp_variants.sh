set -e
cd $GRAFT_REPO_ROOT
for v in base noret; do cp dev/var_$v.so cuda.radixsort_amd/librsort.so; bash dev/kt.sh z_$v --dist zipf; done
