# dev/build_variant.sh NAME "HIPCC FLAGS" [KERNEL SOURCE] -- librsort.so variant with rsort_kernels.hip
# (or a modified copy of it) built with extra flags (lab macros), linked with the library's other
# objects: dev/var_NAME.so. With ALL=1 every library source is compiled with the flags (macros that
# the host code reads too, e.g. a tile shape). On the GPU box, copy it over
# cuda.radixsort_amd/librsort.so (the box's scratch copy) before timing it. Variants that break the
# scatter's offsets can fault the GPU.
set -e
cd /root/repo
python3 cuda.radixsort_amd/build.py > /dev/null
mkdir -p dev/build_var
# (the lab side of the kernels' hooks: dev/lab_hooks.hpp reads the -D switches in $2)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Iinclude -Icuda.radixsort_amd/csrc -DRSORT_LAB_HOOKS=\"../../dev/lab_hooks.hpp\""
/opt/rocm/bin/hipcc $F $2 -c ${3:-cuda.radixsort_amd/csrc/rsort_kernels.hip} -o dev/build_var/$1.o
objs=""
for o in cuda.radixsort_amd/build/*.o; do
    b=$(basename $o .o)
    [ "$b" = rsort_kernels ] && continue
    if [ "${ALL:-0}" = 1 ]; then
        src=$(ls cuda.radixsort_amd/csrc/$b.* | head -1)
        lang=""
        case $src in *.cpp) lang="-x hip" ;; esac
        /opt/rocm/bin/hipcc $F $2 $lang -c $src -o dev/build_var/$1_$b.o
        objs="$objs dev/build_var/$1_$b.o"
    else
        objs="$objs $o"
    fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dev/var_$1.so dev/build_var/$1.o $objs -L/opt/rocm/lib -lrccl
echo dev/var_$1.so
