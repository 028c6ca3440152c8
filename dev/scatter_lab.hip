// Backs DESIGN §3: scatter-kernel variants and ceilings (non-temporal loads/stores, LAB_PAIRS / LAB_K4 / LAB_SHAPE rows, the 4096-key vs 16384-key tiles).
// scatter_lab.hip -- development harness (not part of the library): times variants of the
// fused local-sort + scatter kernel and HBM ceilings on the current GPU, and checks every
// variant's pass output against the first variant's (the pass output is unique).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cuda.radixsort_amd/csrc \
//         dev/scatter_lab.hip -o dev/scatter_lab && dev/scatter_lab [log2n]
#define RSORT_LAB_HOOKS "../../dev/lab_hooks.hpp"
#include "../cuda.radixsort_amd/csrc/rsort_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <vector>

using namespace rsort;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);          \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ void count_mismatch(const uint32_t *a, const uint32_t *b, uint64_t n, unsigned long long *bad) {
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        local += a[i] != b[i];
    if (local) atomicAdd(bad, local);
}

__global__ void copy_dword(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

__global__ void copy_dwordx4(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

struct Ctx {
    uint64_t n;
    uint32_t *keys, *vals, *out, *vout, *ref, *table, *bsums;
    unsigned long long *bad;
    unsigned long long *stamps;
    int cus;
    hipEvent_t e0, e1;
    bool have_ref = false;
};

template <typename F>
float time_ms(Ctx &c, int reps, F f) {
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(c.e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(c.e1, 0));
    CK(hipEventSynchronize(c.e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, c.e0, c.e1));
    return ms / reps;
}

static const char *g_filter = nullptr;

template <int BITS, int THREADS, int KPT, bool PAIRS, typename K>
void run_variant(Ctx &c, const char *name, double wave_mult, K kern, int shift = 0, int reps = 5);

template <int BITS, int THREADS, int KPT, bool PAIRS, int RANK, int MINW>
void variant(Ctx &c, const char *name, double wave_mult, int shift = 0, int reps = 5) {
    run_variant<BITS, THREADS, KPT, PAIRS>(c, name, wave_mult, rs_scatter<BITS, THREADS, KPT, PAIRS, RANK, kDigitShift, MINW>,
                                          shift, reps);
}

// NT: 1 non-temporal loads, 2 non-temporal stores (rs_scatter_lines)
template <int BITS, int THREADS, int KPT, int G, bool PAIRS, int NT = 0>
void lines(Ctx &c, const char *name, double wave_mult, int shift = 0, int reps = 5) {
    run_variant<BITS, THREADS, KPT, PAIRS>(c, name, wave_mult, rs_scatter_lines<BITS, THREADS, KPT, G, PAIRS, kDigitShift, NT>,
                                          shift, reps);
}

template <int BITS, int THREADS, int KPT, bool PAIRS, typename K>
void run_variant(Ctx &c, const char *name, double wave_mult, K kern, int shift, int reps) {
    if (g_filter && !strstr(name, g_filter)) return;
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kern, THREADS, 0));
    const uint64_t T = (uint64_t)THREADS * KPT;
    const uint64_t tiles = (c.n + T - 1) / T;
    const uint64_t target = (uint64_t)(c.cus * bpc * wave_mult);
    const uint64_t tpc = (tiles + target - 1) / target;
    const uint64_t chunks = (tiles + tpc - 1) / tpc;
    HistArgs h{};
    h.keys = c.keys;
    h.table = c.table;
    h.n = c.n;
    h.chunk_keys = tpc * T;
    h.num_chunks = (uint32_t)chunks;
    h.shift = shift;
    h.vec = 1;
    h.split = 1;
    CK(launch_histogram(BITS, kDigitShift, h, 0));
    ScanArgs s{};
    s.table = c.table;
    s.block_sums = c.bsums;
    s.m = (uint64_t)chunks << BITS;
    s.nblocks = (uint32_t)((s.m + kScanSegment - 1) / kScanSegment);
    CK(launch_scan(s, 0));
    ScatterArgs a{};
    a.kin = c.keys;
    a.vin = c.vals;
    a.kout = c.out;
    a.vout = c.vout;
    a.table = c.table;
    a.n = c.n;
    a.chunk_keys = tpc * T;
    a.num_chunks = (uint32_t)chunks;
    a.shift = shift;
    a.stamps = c.stamps;
    CK(hipMemset(c.out, 0, c.n * 4));
    const float ms = time_ms(c, reps, [&] { kern<<<chunks, THREADS>>>(a); });
    CK(hipGetLastError());
    unsigned long long bad = 0;
    if (!c.have_ref) {
        CK(hipMemcpy(c.ref, c.out, c.n * 4, hipMemcpyDeviceToDevice));
        c.have_ref = true;
    } else {
        CK(hipMemset(c.bad, 0, 8));
        count_mismatch<<<4096, 256>>>(c.out, c.ref, c.n, c.bad);
        CK(hipMemcpy(&bad, c.bad, 8, hipMemcpyDeviceToHost));
    }
    const double bytes = (PAIRS ? 16.0 : 8.0) * c.n;
    printf("%-34s bpc=%d tpc=%-5llu chunks=%-6llu %8.3f ms  %7.1f GB/s  %5.1f%%  mismatch=%llu\n", name, bpc,
           (unsigned long long)tpc, (unsigned long long)chunks, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0, bad);
    fflush(stdout);
}

// histogram geometry: THREADS per workgroup, `split` workgroups per chunk, `chunks` chunks
template <int THREADS, int NT = 0, int SUB = 1>
void hist_variant(Ctx &c, const char *name, uint32_t chunks, uint32_t split) {
    if (g_filter && !strstr(name, g_filter)) return;
    HistArgs h{};
    h.keys = c.keys;
    h.table = c.table;
    h.n = c.n;
    h.chunk_keys = (c.n + chunks - 1) / chunks;
    h.chunk_keys = (h.chunk_keys + 16383) / 16384 * 16384;
    h.num_chunks = chunks;
    h.shift = 8;
    h.vec = 1;
    h.split = split;
    const float ms = time_ms(c, 5, [&] {
        hipMemsetAsync(c.table, 0, (size_t)chunks * 256 * 4, 0);
        rs_histogram<8, THREADS, kDigitShift, NT, SUB><<<chunks * split, THREADS>>>(h);
    });
    printf("%-34s grid=%-6u %8.3f ms  %7.1f GB/s (read)\n", name, chunks * split, ms, 4.0 * c.n / ms / 1e6);
    fflush(stdout);
}

int main(int argc, char **argv) {
    Ctx c{};
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    g_filter = argc > 2 ? argv[2] : nullptr;
    c.n = (1ull << lg) - (argc > 3 ? strtoull(argv[3], nullptr, 10) : 0ull);
    CK(hipDeviceGetAttribute(&c.cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&c.keys, c.n * 4));
    CK(hipMalloc(&c.vals, c.n * 4));
    CK(hipMalloc(&c.out, c.n * 4));
    CK(hipMalloc(&c.vout, c.n * 4));
    CK(hipMalloc(&c.ref, c.n * 4));
    CK(hipMalloc(&c.table, (c.n / 1024 + 65536) * 4 * 16));
    CK(hipMalloc(&c.bsums, 1 << 24));
    CK(hipMalloc(&c.bad, 8));
    CK(hipMalloc(&c.stamps, 65536 * 8 * 8));
    CK(hipEventCreate(&c.e0));
    CK(hipEventCreate(&c.e1));
    CK(launch_gen_uniform(c.keys, c.n, 0x5EED, 0));
    if (getenv("LAB_ZIPF")) {  // Zipf(1.0) over 2^20 ranks, key = fmix32(rank) (== rsort_gen_zipf)
        const uint64_t ranks = 1u << 20;
        std::vector<double> cum(ranks);
        double acc = 0;
        for (uint64_t r = 0; r < ranks; ++r) cum[r] = (acc += 1.0 / (double)(r + 1));
        std::vector<uint32_t> cdf(ranks);
        for (uint64_t r = 0; r < ranks; ++r) {
            const double t = floor(cum[r] / acc * 4294967296.0);
            cdf[r] = (uint32_t)(t > 4294967295.0 ? 4294967295.0 : t);
        }
        cdf[ranks - 1] = 4294967295u;
        uint32_t *dcdf;
        CK(hipMalloc(&dcdf, ranks * 4));
        CK(hipMemcpy(dcdf, cdf.data(), ranks * 4, hipMemcpyHostToDevice));
        CK(launch_gen_zipf(c.keys, c.n, 0x5EED, dcdf, ranks, 0));
        printf("keys: zipf\n");
    }
    CK(launch_gen_iota(c.vals, c.n, 0, 0));
    CK(hipDeviceSynchronize());
    printf("n=%llu cus=%d\n", (unsigned long long)c.n, c.cus);

    if (!g_filter) {
        const float ms1 = time_ms(c, 5, [&] { copy_dword<<<c.cus * 8, 256>>>(c.keys, c.out, c.n); });
        const float ms4 = time_ms(c, 5, [&] { copy_dwordx4<<<c.cus * 8, 256>>>((const uint4 *)c.keys, (uint4 *)c.out, c.n / 4); });
        const float ms4b = time_ms(c, 5, [&] { copy_dwordx4<<<c.cus * 32, 256>>>((const uint4 *)c.keys, (uint4 *)c.out, c.n / 4); });
        printf("copy dword   %8.3f ms %7.1f GB/s\n", ms1, 8.0 * c.n / ms1 / 1e6);
        printf("copy dwordx4 %8.3f ms %7.1f GB/s\n", ms4, 8.0 * c.n / ms4 / 1e6);
        printf("copy dwordx4 (32/CU) %8.3f ms %7.1f GB/s\n", ms4b, 8.0 * c.n / ms4b / 1e6);
    }
#ifdef LINES_ONLY
    // -DLINES_ONLY: just the line-combining kernels (fast rebuilds); phase stamps of the line kernel
    // live in dev/lines_exp.hip (-DLX_STAMPS)
    if (getenv("LAB_K4")) {
        variant<4, 512, 16, false, kRankAtomic, 4>(c, "k4 512x16 atomic w4 (lib)", 1.0);
        lines<4, 256, 16, 32, false, 3>(c, "k4 256x16 lines32 nt", 1.0);
        lines<4, 256, 16, 32, false, 1>(c, "k4 256x16 lines32 ntload", 1.0);
        lines<4, 256, 16, 32, false, 3>(c, "k4 256x16 lines32 nt again", 1.0);
        lines<4, 1024, 16, 32, false, 3>(c, "k4 1024x16 lines32 nt", 1.0);
        lines<4, 1024, 16, 32, false, 3>(c, "k4 1024x16 lines32 nt again", 1.0);
        c.have_ref = false;
        variant<3, 512, 16, false, kRankAtomic, 4>(c, "k3 512x16 atomic w4 (lib)", 1.0);
        lines<3, 256, 16, 32, false, 3>(c, "k3 256x16 lines32 nt", 1.0);
        c.have_ref = false;
        variant<2, 512, 16, false, kRankAtomic, 4>(c, "k2 512x16 atomic w4 (lib)", 1.0);
        lines<2, 256, 16, 32, false, 3>(c, "k2 256x16 lines32 nt", 1.0);
        return 0;
    }
    if (getenv("LAB_P1")) {  // keys as pass 1 sees them: pass 0's output, then a pass on digit 1
        lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt (pass 0)", 1.0);
        CK(hipMemcpy(c.keys, c.out, c.n * 4, hipMemcpyDeviceToDevice));
        c.have_ref = false;
        printf("input: pass-0 output\n");
        lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt (pass 1)", 1.0, 8);
        lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt (pass 1) again", 1.0, 8);
        return 0;
    }
    if (getenv("LAB_SHAPE")) {  // keys-only line kernel: 16384-key tiles as 1024x16 or 512x32
        lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt", 1.0);
        lines<8, 512, 32, 32, false, 3>(c, "k8 512x32 lines32 nt", 1.0);
        lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt again", 1.0);
        lines<8, 512, 32, 32, false, 3>(c, "k8 512x32 lines32 nt again", 1.0);
        return 0;
    }
    if (getenv("LAB_PAIRS2")) {  // key+value line kernel shape: 512 x 16 or 1024 x 8 (nt stores)
        lines<8, 512, 16, 16, true, 2>(c, "k8 pairs 512x16 lines16 ntstore", 1.0);
        lines<8, 1024, 8, 16, true, 2>(c, "k8 pairs 1024x8 lines16 ntstore", 1.0);
        lines<8, 512, 16, 16, true, 2>(c, "k8 pairs 512x16 lines16 ntstore again", 1.0);
        lines<8, 1024, 8, 16, true, 2>(c, "k8 pairs 1024x8 lines16 ntstore again", 1.0);
        return 0;
    }
    if (getenv("LAB_PAIRS")) {  // key+value line kernel: non-temporal loads / stores
        lines<8, 512, 16, 16, true, 0>(c, "k8 pairs 512x16 lines16", 1.0);
        lines<8, 512, 16, 16, true, 1>(c, "k8 pairs 512x16 lines16 ntload", 1.0);
        lines<8, 512, 16, 16, true, 3>(c, "k8 pairs 512x16 lines16 nt", 1.0);
        lines<8, 512, 16, 16, true, 2>(c, "k8 pairs 512x16 lines16 ntstore", 1.0);
        lines<8, 512, 16, 16, true, 0>(c, "k8 pairs 512x16 lines16 again", 1.0);
        lines<8, 512, 16, 16, true, 3>(c, "k8 pairs 512x16 lines16 nt again", 1.0);
        return 0;
    }
    lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt", 1.0);
    return 0;
#endif
    hist_variant<256>(c, "hist 256 x8", 256, 8);
    hist_variant<512>(c, "hist 512 x8", 256, 8);
    hist_variant<1024>(c, "hist 1024 x4", 256, 4);
    hist_variant<1024>(c, "hist 1024 x8", 256, 8);
    constexpr int CT = kRankCount;
    constexpr int AT = kRankAtomic;
    variant<8, 512, 16, false, AT, 0>(c, "k8 512x16 atomic (rs_scatter)", 1.0);
    variant<8, 512, 16, false, CT, 0>(c, "k8 512x16 ballot (rs_scatter)", 1.0);
    lines<8, 1024, 16, 32, false, 3>(c, "k8 1024x16 lines32 nt (lib)", 1.0);
    c.have_ref = false;
    variant<8, 512, 16, true, AT, 0>(c, "k8 pairs 512x16 atomic (rs_scatter)", 1.0);
    lines<8, 512, 16, 16, true, 2>(c, "k8 pairs 512x16 lines16 ntstore (lib)", 1.0);
    c.have_ref = false;
    variant<4, 512, 16, false, AT, 4>(c, "k4 512x16 atomic w4", 1.0);
    lines<4, 256, 16, 32, false, 3>(c, "k4 256x16 lines32 nt (lib)", 1.0);
    lines<4, 1024, 16, 32, false, 3>(c, "k4 1024x16 lines32 nt (lib, n >= 2^28)", 1.0);
    return 0;
}
