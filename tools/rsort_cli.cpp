// rsort_cli.cpp -- the reference's harness (SourceCode/Parallel7.cu:664-775), on the MI355X library.
//
//   rsort_cli [blockSize [numBits]] [--debug] [--n N]
//
// Same flow and output as the reference main: device info, input of n = (1 << 24) + 1 glibc
// rand() keys (DEBUG: n = 513, rand() & 0xFF, numBits = 4, arrays printed), then sort by host,
// by "Thrust" (rocPRIM on ROCm) and by device through include/radixsort.hpp, each checked
// against the host result ("CORRECT :)" / "INCORRECT :("). Exit status is 0 like the reference
// (P7:774) unless --strict is given, in which case an incorrect result exits 1.
//
// sortByHost below is the harness's own host sort (the reference defines it in every source
// file; Baseline1.cu:15-64 semantics). It is the checker of this tool only; librsort.so has no
// host sort and never falls back to one.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "radixsort.hpp"

void sortByHost(const uint32_t *in, int n, uint32_t *out, int nBits) {
    const int nBins = 1 << nBits;
    std::vector<int> hist(nBins);
    std::vector<uint32_t> buf(in, in + n);
    uint32_t *src = buf.data(), *dst = out;
    for (int bit = 0; bit < 32; bit += nBits) {
        std::fill(hist.begin(), hist.end(), 0);
        for (int i = 0; i < n; ++i) hist[(src[i] >> bit) & (nBins - 1)]++;
        int run = 0;
        for (int b = 0; b < nBins; ++b) {
            const int c = hist[b];
            hist[b] = run;
            run += c;
        }
        for (int i = 0; i < n; ++i) dst[hist[(src[i] >> bit) & (nBins - 1)]++] = src[i];
        uint32_t *t = src;
        src = dst;
        dst = t;
    }
    if (src != out) memcpy(out, src, (size_t)n * sizeof(uint32_t));
}

static void printDeviceInfo() {
    hipDeviceProp_t p;
    RSORT_CHECK(hipGetDeviceProperties(&p, 0) == hipSuccess ? RSORT_OK : RSORT_ERR_HIP);
    printf("**********GPU info**********\n");
    printf("Name: %s\n", p.name);
    printf("Compute capability: %d.%d (%s)\n", p.major, p.minor, p.gcnArchName);
    printf("Num SMs: %d\n", p.multiProcessorCount);
    printf("Max num threads per SM: %d\n", p.maxThreadsPerMultiProcessor);
    printf("Max num warps per SM: %d\n", p.maxThreadsPerMultiProcessor / p.warpSize);
    printf("GMEM: %zu byte\n", p.totalGlobalMem);
    printf("SMEM per SM: %zu byte\n", p.maxSharedMemoryPerMultiProcessor);
    printf("SMEM per block: %zu byte\n", p.sharedMemPerBlock);
    printf("****************************\n");
}

static bool checkCorrectness(const uint32_t *out, const uint32_t *correct, int n) {
    for (int i = 0; i < n; ++i)
        if (out[i] != correct[i]) {
            printf("INCORRECT :(\n");
            return false;
        }
    printf("CORRECT :)\n");
    return true;
}

static void printArray(const uint32_t *a, int n) {
    for (int i = 0; i < n; ++i) printf("%u ", a[i]);
    printf("\n");
}

int main(int argc, char **argv) {
    bool debug = false, strict = false;
    long long n_arg = -1;
    std::vector<const char *> pos;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--debug")) debug = true;
        else if (!strcmp(argv[i], "--strict")) strict = true;
        else if (!strcmp(argv[i], "--n") && i + 1 < argc) n_arg = atoll(argv[++i]);
        else pos.push_back(argv[i]);
    }
    RSORT_CHECK(hipSetDevice(0) == hipSuccess ? RSORT_OK : RSORT_ERR_NODEV);
    printDeviceInfo();

    const int n = n_arg > 0 ? (int)n_arg : (debug ? 513 : (1 << 24) + 1);
    printf("\nInput size: %d\n", n);
    std::vector<uint32_t> input(n), output(n), correct(n);
    for (int i = 0; i < n; ++i) input[i] = debug ? ((uint32_t)rand() & 0xFFu) : (uint32_t)rand();
    if (debug) printArray(input.data(), n);

    int blockSize = 512;
    if (pos.size() > 0) blockSize = atoi(pos[0]);
    printf("Block size: %d\n", blockSize);
    int numBits = debug ? 4 : 8;
    if (pos.size() > 1) numBits = atoi(pos[1]);
    printf("Digit width: %d-bit\n", numBits);

    sort(input.data(), n, correct.data(), SORT_BY_HOST, numBits);
    if (debug) printArray(correct.data(), n);

    bool ok = true;
    memset(output.data(), 0, (size_t)n * 4);
    sort(input.data(), n, output.data(), SORT_BY_THRUST);
    if (debug) printArray(output.data(), n);
    ok &= checkCorrectness(output.data(), correct.data(), n);

    memset(output.data(), 0, (size_t)n * 4);
    sort(input.data(), n, output.data(), SORT_BY_DEVICE, numBits, blockSize);
    if (debug) printArray(output.data(), n);
    ok &= checkCorrectness(output.data(), correct.data(), n);
    return (strict && !ok) ? 1 : EXIT_SUCCESS;
}
