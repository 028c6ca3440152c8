#!/usr/bin/env bash
# build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference's own sequential sorts into oracle/_ref/libref.so, straight
# from the unmodified sources under /root/reference (read-only; never copied into the repo):
#   sortByHost                        SourceCode/Baseline1.cu:15-64
#   sortByHostUsingParallelAlgorithm  SourceCode/Baseline4.cu:67-273
# Each function is cut out of its .cu by line range (the rest of those files needs the
# CUDA toolkit and Thrust, which this image does not have) and piped to g++ on stdin, so
# no reference text is ever written to disk. The first line of each range is checked
# against the expected signature so a moved reference fails loudly instead of building
# the wrong code. Baseline4's phase timers are compiled out with
# -DMEASURE_PORTION_EXECUTION_TIME=0 (the reference's own switch, Baseline4.cu:12).
#
# Output: oracle/_ref/libref.so (git-ignored; travels to the GPU box with the snapshot).
# Exit 0 and build nothing when /root/reference is absent (the GPU box).
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
ref="${RSORT_REFERENCE_DIR:-/root/reference}/SourceCode"
out="$here/_ref"
if [[ ! -d "$ref" ]]; then
    echo "build_ref: $ref absent -- keeping prebuilt oracle/_ref (if any)"
    exit 0
fi
mkdir -p "$out"

extract() {  # file first last expected-prefix
    local first_line
    first_line="$(sed -n "${2}p" "$ref/$1")"
    if [[ "$first_line" != "$4"* ]]; then
        echo "build_ref: $1:$2 is '$first_line', expected '$4...'" >&2
        exit 1
    fi
    sed -n "${2},${3}p" "$ref/$1"
}

hdrs=(-include stdio.h -include stdint.h -include stdlib.h -include string.h)
extract Baseline1.cu 15 64 "void sortByHost(const uint32_t * in, int n, uint32_t * out, int nBits)" |
    g++ -O2 -fPIC -x c++ "${hdrs[@]}" -c - -o "$out/baseline1.o"
extract Baseline4.cu 67 273 "void sortByHostUsingParallelAlgorithm(" |
    g++ -O2 -fPIC -x c++ "${hdrs[@]}" -DMEASURE_PORTION_EXECUTION_TIME=0 -c - -o "$out/baseline4.o"
g++ -O2 -fPIC -c "$here/ref_shim.cpp" -o "$out/ref_shim.o"
g++ -shared -o "$out/libref.so" "$out/baseline1.o" "$out/baseline4.o" "$out/ref_shim.o"
rm -f "$out"/*.o
echo "build_ref: built $out/libref.so"
