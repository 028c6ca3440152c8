// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// C-linkage entry points around the reference's own host functions, which
// oracle/build_ref.sh compiles straight from the unmodified sources under
// /root/reference (line ranges checked there). No reference text lives in this repo:
// this file only declares the two reference functions and forwards to them.
//
//   sortByHost                        SourceCode/Baseline1.cu:15-64
//   sortByHostUsingParallelAlgorithm  SourceCode/Baseline4.cu:67-273
#include <stdint.h>

void sortByHost(const uint32_t *in, int n, uint32_t *out, int nBits);
void sortByHostUsingParallelAlgorithm(const uint32_t *input, int n, uint32_t *output,
                                      int numBits, int blockSize);

extern "C" __attribute__((visibility("default"))) void ref_sort_by_host(const uint32_t *in, int n,
                                                                        uint32_t *out, int nbits) {
    sortByHost(in, n, out, nbits);
}

extern "C" __attribute__((visibility("default"))) void ref_block_sort(const uint32_t *in, int n,
                                                                      uint32_t *out, int nbits,
                                                                      int block) {
    sortByHostUsingParallelAlgorithm(in, n, out, nbits, block);
}
