# dev/build_variant.sh NAME "HIPCC FLAGS" [KERNEL SOURCE] -- librsort.so variant with rsort_kernels.hip
# (or a modified copy of it) built with extra flags (lab macros), linked with the library's other
# objects: dev/var_NAME.so. On the GPU box, copy it over cuda.radixsort_amd/librsort.so (the box's
# scratch copy) before timing it. Variants that break the scatter's offsets can fault the GPU.
set -e
cd /root/repo
python3 cuda.radixsort_amd/build.py > /dev/null
mkdir -p dev/build_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Iinclude -Icuda.radixsort_amd/csrc $2 \
    -c ${3:-cuda.radixsort_amd/csrc/rsort_kernels.hip} -o dev/build_var/$1.o
objs=$(ls cuda.radixsort_amd/build/*.o | grep -v rsort_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dev/var_$1.so dev/build_var/$1.o $objs -L/opt/rocm/lib -lrccl
echo dev/var_$1.so
