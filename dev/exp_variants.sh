# dev/exp_variants.sh V1 V2 ... -- kernel traces of the Zipf-keys and all-equal benches for each
# library variant dev/var_V.so (dev/build_variant.sh), copied over the box's librsort.so in turn
set -e
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  cp dev/var_$v.so cuda.radixsort_amd/librsort.so
  bash dev/kt.sh z_$v --dist zipf
  bash dev/kt.sh e_$v --dist equal
done
