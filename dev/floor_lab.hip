// Backs DESIGN §3 "Floors" (round 6): one pass of each production scatter kernel,
// timed on uniform input, built twice -- as the library builds it, and with its output stores compiled out
// (-DRSORT_LAB_NO_STORES through dev/lab_hooks.hpp: the values that would be stored are kept live, so every
// LDS read stays). The no-store time is the pass's LDS / VALU floor; the gap between it and the stored pass
// is what the write stream adds.
//   c4   rs_scatter_pairs<8, 1024, 8, 1>: 2^30 key + value pairs, 8192-pair tiles, 256 chunks
//   c3   rs_scatter_lines<8, 1024, 16, 32, false, 0, 3>: 2^30 keys, 16384-key tiles, 256 chunks
//   c2   rs_scatter_lines<4, 256, 16, 32, false, 0, 1>: 2^26 keys, 4096-key tiles, 1024 chunks (4 per CU),
//        a middle pass (next-digit counts on) and the last pass (off)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cuda.radixsort_amd/csrc dev/floor_lab.hip -o dev/floor_lab
//   hipcc ... -DRSORT_LAB_NO_STORES dev/floor_lab.hip -o dev/floor_lab_ns
//   dev/floor_lab [reps = 10]   (JSON lines)
#define RSORT_LAB_HOOKS "../../dev/lab_hooks.hpp"
#include "../cuda.radixsort_amd/csrc/rsort_kernels.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

using namespace rsort;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

#ifdef RSORT_LAB_NO_STORES
static const char *kBuild = "no_stores";
#else
static const char *kBuild = "stores";
#endif

static hipEvent_t e0, e1;

template <class F>
static double best_of(int reps, int rounds, F f) {
    f();
    CK(hipDeviceSynchronize());
    double best = 1e30;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, (double)ms / reps);
    }
    return best;
}

// the chunk table of `keys` at `shift` (histogram + scan), as the library's fixed-chunk passes have it
template <int BITS>
static void table_for(const uint32_t *keys, uint64_t n, uint32_t shift, uint32_t *table, uint64_t chunk_keys,
                      uint32_t chunks, uint32_t *bsums) {
    HistArgs h{};
    h.keys = keys;
    h.table = table;
    h.n = n;
    h.chunk_keys = chunk_keys;
    h.num_chunks = chunks;
    h.shift = shift;
    h.vec = 1;
    h.split = 1;
    rs_histogram<BITS, 1024, kDigitShift, 1, 8><<<chunks, 1024>>>(h);
    ScanArgs sa{};
    sa.table = table;
    sa.block_sums = bsums;
    sa.m = (uint64_t)(1u << BITS) * chunks;
    sa.nblocks = (uint32_t)((sa.m + kScanSegment - 1) / kScanSegment);
    rs_scan_reduce<<<sa.nblocks, kScanThreads>>>(sa);
    rs_scan_down<<<sa.nblocks, kScanThreads>>>(sa);
    CK(hipGetLastError());
}

static void line(const char *what, uint64_t n, double bytes_per_key, double ms) {
    printf("{\"build\": \"%s\", \"pass\": \"%s\", \"keys\": %llu, \"ms\": %.4f, \"frac_of_8TBs\": %.4f}\n", kBuild, what,
           (unsigned long long)n, ms, bytes_per_key * n / (ms * 1e-3) / 8e12);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t N = 1ull << 30;
    uint32_t *k0, *v0, *k1, *v1, *table, *bsums, *next;
    CK(hipMalloc(&k0, N * 4));
    CK(hipMalloc(&v0, N * 4));
    CK(hipMalloc(&k1, N * 4));
    CK(hipMalloc(&v1, N * 4));
    CK(hipMalloc(&table, 1u << 22));
    CK(hipMalloc(&next, 1u << 22));
    CK(hipMalloc(&bsums, 1u << 16));
    rs_gen_uniform<<<65536, 256>>>(k0, N, 0x5EED);
    rs_gen_iota<<<65536, 256>>>(v0, N, 0);
    CK(hipDeviceSynchronize());
    auto args = [&](uint64_t n, uint64_t chunk_keys, uint32_t chunks) {
        ScatterArgs a{};
        a.kin = k0;
        a.vin = v0;
        a.kout = k1;
        a.vout = v1;
        a.table = table;
        a.n = n;
        a.chunk_keys = chunk_keys;
        a.num_chunks = chunks;
        a.shift = 0;
        return a;
    };
    {  // C4's pass: 8192-pair tiles, 256 chunks
        const uint64_t T = 8192, tiles = N / T, tpc = tiles / 256;
        table_for<8>(k0, N, 0, table, tpc * T, 256, bsums);
        const ScatterArgs a = args(N, tpc * T, 256);
        line("c4_pairs_pass", N, 16, best_of(reps, 3, [&] { rs_scatter_pairs<8, 1024, 8, 1><<<256, 1024>>>(a); }));
    }
    {  // C3's pass: 16384-key tiles, 256 chunks
        const uint64_t T = 16384, tiles = N / T, tpc = tiles / 256;
        table_for<8>(k0, N, 0, table, tpc * T, 256, bsums);
        const ScatterArgs a = args(N, tpc * T, 256);
        line("c3_keys_pass", N, 8, best_of(reps, 3, [&] {
                 rs_scatter_lines<8, 1024, 16, kLineKeys, false, kDigitShift, 3><<<256, 1024>>>(a);
             }));
    }
    {  // C2's passes: 2^26 keys, 4096-key tiles, 1024 chunks (four 256-thread workgroups per CU)
        const uint64_t n = 1ull << 26, T = 4096, tiles = n / T, chunks = 1024, tpc = tiles / chunks;
        table_for<4>(k0, n, 0, table, tpc * T, (uint32_t)chunks, bsums);
        ScatterArgs a = args(n, tpc * T, (uint32_t)chunks);
        line("c2_keys_last_pass", n, 8, best_of(reps * 4, 3, [&] {
                 rs_scatter_lines<4, 256, 16, kLineKeys, false, kDigitShift, 1><<<(unsigned)chunks, 256>>>(a);
             }));
        CK(hipMemset(next, 0, 16 * chunks * 4));
        a.next_table = next;  // next-digit counts on (no tail scan: done == nullptr)
        line("c2_keys_middle_pass", n, 8, best_of(reps * 4, 3, [&] {
                 rs_scatter_lines<4, 256, 16, kLineKeys, false, kDigitShift, 1><<<(unsigned)chunks, 256>>>(a);
             }));
        // the same middle pass as a sort runs it: its offsets from the raw next-digit counts the pass before
        // added (every workgroup sums the whole 16 x 1024 table, raw_offsets), on that pass's output. Pass 0
        // (k0 -> k1) counts digit 1 into `next`; pass 1 (k1, shift 4) then reads `next` raw, counts into t2,
        // clears t3 (the tables stay consistent with k1 on every repeat: only t2 accumulates)
#ifndef RSORT_LAB_NO_STORES
        uint32_t *t2, *t3;
        CK(hipMalloc(&t2, 16 * chunks * 4));
        CK(hipMalloc(&t3, 16 * chunks * 4));
        CK(hipMemset(next, 0, 16 * chunks * 4));
        CK(hipMemset(t2, 0, 16 * chunks * 4));
        ScatterArgs p0 = a;
        p0.next_table = next;
        rs_scatter_lines<4, 256, 16, kLineKeys, false, kDigitShift, 1><<<(unsigned)chunks, 256>>>(p0);
        CK(hipDeviceSynchronize());
        ScatterArgs p1 = a;
        p1.kin = k1;
        p1.kout = k0 + (1ull << 27);  // (a buffer of its own, past the C2 input)
        p1.shift = 4;
        p1.table = next;
        p1.raw_table = 1;
        p1.next_table = t2;
        p1.zero_table = t3;
        line("c2_keys_middle_pass_raw_offsets", n, 8, best_of(reps * 4, 3, [&] {
                 rs_scatter_lines<4, 256, 16, kLineKeys, false, kDigitShift, 1><<<(unsigned)chunks, 256>>>(p1);
             }));
        // and with those offsets pre-scanned instead (the pass without raw_offsets, same input and tables)
        CK(hipMemcpy(t3, next, 16 * chunks * 4, hipMemcpyDeviceToDevice));
        ScanArgs sa{};
        sa.table = t3;
        sa.block_sums = bsums;
        sa.m = 16 * chunks;
        sa.nblocks = (uint32_t)((sa.m + kScanSegment - 1) / kScanSegment);
        rs_scan_reduce<<<sa.nblocks, kScanThreads>>>(sa);
        rs_scan_down<<<sa.nblocks, kScanThreads>>>(sa);
        CK(hipDeviceSynchronize());
        ScatterArgs p2 = p1;
        p2.table = t3;
        p2.raw_table = 0;
        p2.zero_table = nullptr;
        line("c2_keys_middle_pass_scanned", n, 8, best_of(reps * 4, 3, [&] {
                 rs_scatter_lines<4, 256, 16, kLineKeys, false, kDigitShift, 1><<<(unsigned)chunks, 256>>>(p2);
             }));
#endif
    }
    return 0;
}
