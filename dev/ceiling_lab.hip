// Backs DESIGN §3 "Ceilings" (round 5): the HBM copy ceiling of this pool's MI355X
// boxes against MI355X_MICROARCH.md's 6.29 TB/s float4 copy, and what per-workgroup rates look like on
// a plain copy (do equal chunks run at unequal rates without any sort work?).
//
// Every variant moves 16-B quads; bytes = read + write. Variants:
//   copy-stride  grid-stride loop, each iteration a workgroup moves THREADS x Q contiguous quads
//   copy-chunk   one contiguous chunk per workgroup (the sort's layout), records per-workgroup start/end,
//                HW_ID and XCC_ID (s_getreg) for the rate-correlation table
//   read / write the two halves alone
//   runs         the k = 8 keys-pass write stream (dev/runlen_lab.hip's `runs`): 16384-key tiles written
//                as 256 runs of 64 keys continuing 256 regions, one chunk per workgroup
// Load / store policy: default or non-temporal (__builtin_nontemporal_*), each side separately.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/ceiling_lab.hip -o dev/ceiling_lab
//   dev/ceiling_lab [log2 keys per buffer = 30] [reps = 10] [pairs | c2]   (JSON lines on stdout; `pairs`: the
//   pairs pass's write-stream floor, runs of 32 pairs in two arrays, beside runs64 -- VERDICT r4 weak #3;
//   `c2`: the C2 pass's write-stream floor, 2^26 keys in runs of 256 into 16 regions -- VERDICT r5 item 3)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// HW_ID (hwreg 4, 32 bits: wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13) and XCC_ID (hwreg 20, 4 bits)
__device__ __forceinline__ uint32_t hw_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 4); }
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((15 << 11) | 20); }

template <int TH, int Q, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void copy_stride(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, uint64_t n4) {
    for (uint64_t b = (uint64_t)blockIdx.x * TH * Q; b < n4; b += (uint64_t)gridDim.x * TH * Q) {
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) v[j] = ld<NTL>(in + b + threadIdx.x + j * TH);
#pragma unroll
        for (int j = 0; j < Q; ++j) st<NTS>(out + b + threadIdx.x + j * TH, v[j]);
    }
}

// rec (nullable): per workgroup {t0, t1, hw_id, xcc_id}
template <int TH, int Q, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void copy_chunk(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, uint64_t chunk4,
                                                 unsigned long long *rec) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t beg = (uint64_t)blockIdx.x * chunk4, end = beg + chunk4;
    for (uint64_t b = beg; b < end; b += TH * Q) {
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) v[j] = ld<NTL>(in + b + threadIdx.x + j * TH);
#pragma unroll
        for (int j = 0; j < Q; ++j) st<NTS>(out + b + threadIdx.x + j * TH, v[j]);
    }
    if (rec) {
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long *p = rec + 4 * blockIdx.x;
            p[0] = t0;
            p[1] = __builtin_amdgcn_s_memrealtime();
            p[2] = hw_id();
            p[3] = xcc_id();
        }
    }
}

template <int TH, int Q, bool NTL>
__global__ __launch_bounds__(TH) void read_only(const u32x4 *__restrict__ in, uint32_t *__restrict__ sink, uint64_t n4) {
    uint32_t acc = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * TH * Q; b < n4; b += (uint64_t)gridDim.x * TH * Q) {
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) v[j] = ld<NTL>(in + b + threadIdx.x + j * TH);
#pragma unroll
        for (int j = 0; j < Q; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;  // never in practice; keeps the loads
}

template <int TH, int Q, bool NTS>
__global__ __launch_bounds__(TH) void write_only(u32x4 *__restrict__ out, uint64_t n4) {
    const u32x4 v = {blockIdx.x, threadIdx.x, 1u, 2u};
    for (uint64_t b = (uint64_t)blockIdx.x * TH * Q; b < n4; b += (uint64_t)gridDim.x * TH * Q) {
#pragma unroll
        for (int j = 0; j < Q; ++j) st<NTS>(out + b + threadIdx.x + j * TH, v);
    }
}

// the keys pass's write stream: tile of TH*Q*4 keys -> 256 runs of T/256 keys, run r continuing region r
template <int TH, int Q, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void runs(const u32x4 *__restrict__ in, uint32_t *__restrict__ out, uint64_t n,
                                           uint32_t tpc) {
    constexpr uint32_t T = TH * Q * 4, L = T / 256;
    const uint64_t region = n / 256 - 32;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) v[j] = ld<NTL>(reinterpret_cast<const u32x4 *>(in) + tb / 4 + threadIdx.x + j * TH);
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const uint32_t i = (threadIdx.x + j * TH) * 4;
            const uint64_t pos = (i / L) * region + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            st<NTS>(reinterpret_cast<u32x4 *>(out + pos), v[j]);
        }
    }
}

// the pairs pass's write stream (rs_scatter_pairs' shape): tile of TH*Q*4 pairs read from two arrays and
// written to two as 256 runs of T/256 pairs (128-B lines at 8192-pair tiles) continuing 256 regions each
template <int TH, int Q, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void runs_pairs(const u32x4 *__restrict__ ink, const u32x4 *__restrict__ inv,
                                                 uint32_t *__restrict__ outk, uint32_t *__restrict__ outv, uint64_t n,
                                                 uint32_t tpc) {
    constexpr uint32_t T = TH * Q * 4, L = T / 256;
    const uint64_t region = n / 256 - 32;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 k[Q], v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            k[j] = ld<NTL>(ink + tb / 4 + threadIdx.x + j * TH);
            v[j] = ld<NTL>(inv + tb / 4 + threadIdx.x + j * TH);
        }
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const uint32_t i = (threadIdx.x + j * TH) * 4;
            const uint64_t pos = (i / L) * region + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            st<NTS>(reinterpret_cast<u32x4 *>(outk + pos), k[j]);
            st<NTS>(reinterpret_cast<u32x4 *>(outv + pos), v[j]);
        }
    }
}

// the k = 4 keys pass's write stream (C2): tiles of TH*Q*4 keys written as RG runs of
// T/RG keys, run r continuing region r; one chunk of tpc tiles per workgroup (C2: 4096-key tiles, 16 regions,
// runs of 256 keys, 1024 chunks = 4 workgroups per CU)
template <int TH, int Q, int RG, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void runs_rg(const u32x4 *__restrict__ in, uint32_t *__restrict__ out, uint64_t n,
                                              uint32_t tpc) {
    constexpr uint32_t T = TH * Q * 4, L = T / RG;
    const uint64_t region = n / RG - 32;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) v[j] = ld<NTL>(in + tb / 4 + threadIdx.x + j * TH);
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const uint32_t i = (threadIdx.x + j * TH) * 4;
            const uint64_t pos = (i / L) * region + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            st<NTS>(reinterpret_cast<u32x4 *>(out + pos), v[j]);
        }
    }
}

// runs64 variants that separate the two sides of the pairs stream's advantage: SPLITR reads each tile as
// two halves from the two halves of the input (two read streams per workgroup, like keys + values);
// SPLITW writes the odd digits' runs into a second array (two write arrays, like the pairs stream)
template <int TH, int Q, bool SPLITR, bool SPLITW>
__global__ __launch_bounds__(TH) void runs_split(const u32x4 *__restrict__ in, uint32_t *__restrict__ out,
                                                 uint32_t *__restrict__ out2, uint64_t n, uint32_t tpc) {
    constexpr uint32_t T = TH * Q * 4, L = T / 256;
    const uint64_t region = n / 256 - 32;
    const uint64_t half4 = n / 8;  // quads per input half
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 v[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            uint64_t qi = tb / 4 + threadIdx.x + j * TH;
            if (SPLITR) qi = (j & 1) ? half4 + tb / 8 + threadIdx.x + (j / 2) * TH : tb / 8 + threadIdx.x + (j / 2) * TH;
            v[j] = ld<true>(in + qi);
        }
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const uint32_t i = (threadIdx.x + j * TH) * 4;
            const uint32_t r = i / L;
            const uint64_t pos = (SPLITW ? (r / 2) : r) * region + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            st<true>(reinterpret_cast<u32x4 *>(((SPLITW && (r & 1)) ? out2 : out) + pos), v[j]);
        }
    }
}

static hipEvent_t e0, e1;
static int g_reps = 10;

template <class F>
static double timeit(F f) {
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < g_reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / g_reps;
}

static void line(const char *kind, const char *mode, int th, int q, int grid_per_cu, int ntl, int nts, double bytes,
                 double ms) {
    printf("{\"kind\": \"%s\", \"mode\": \"%s\", \"threads\": %d, \"quads_per_thread\": %d, \"grid_per_cu\": %d, "
           "\"nt_loads\": %d, \"nt_stores\": %d, \"bytes\": %.0f, \"ms\": %.4f, \"TBs\": %.3f}\n",
           kind, mode, th, q, grid_per_cu, ntl, nts, bytes, ms, bytes / ms / 1e9);
    fflush(stdout);
}

template <int TH, int Q, bool NTL, bool NTS>
static void stride_set(const u32x4 *a, u32x4 *b, uint64_t n4, int cus, const char *label) {
    for (int g : {1, 2, 4, 8, 16, 32}) {
        if (TH == 1024 && g > 16) continue;
        const double ms = timeit([&] { copy_stride<TH, Q, NTL, NTS><<<cus * g, TH>>>(a, b, n4); });
        line("copy", label, TH, Q, g, NTL, NTS, 32.0 * n4, ms);
    }
}

// per-workgroup record of one copy-chunk launch: end spread and duration by XCC / SE / CU
static void chunk_rates(const char *label, std::vector<unsigned long long> &h, int nwg) {
    std::vector<double> dur(nwg);
    unsigned long long t0min = ~0ull, t1min = ~0ull, t1max = 0, t0max = 0;
    for (int i = 0; i < nwg; ++i) {
        dur[i] = (double)(h[4 * i + 1] - h[4 * i]) * 0.01;  // 100 MHz -> us
        t0min = std::min(t0min, h[4 * i]);
        t0max = std::max(t0max, h[4 * i]);
        t1min = std::min(t1min, h[4 * i + 1]);
        t1max = std::max(t1max, h[4 * i + 1]);
    }
    std::vector<double> s = dur;
    std::sort(s.begin(), s.end());
    double xs[16] = {0}, xn[16] = {0}, xmin[16], xmax[16];
    for (int x = 0; x < 16; ++x) xmin[x] = 1e30, xmax[x] = 0;
    double se_s[8] = {0}, se_n[8] = {0};
    int bad_rr = 0;
    for (int i = 0; i < nwg; ++i) {
        const int x = (int)(h[4 * i + 3] & 15u);
        const int se = (int)((h[4 * i + 2] >> 13) & 7u);
        xs[x] += dur[i];
        xn[x] += 1;
        xmin[x] = std::min(xmin[x], dur[i]);
        xmax[x] = std::max(xmax[x], dur[i]);
        se_s[se] += dur[i];
        se_n[se] += 1;
        if (x != i % 8) ++bad_rr;
    }
    printf("{\"kind\": \"chunk_rates\", \"mode\": \"%s\", \"workgroups\": %d, \"wall_us\": %.1f, \"start_spread_us\": %.1f, "
           "\"end_spread_us\": %.1f, \"dur_us_min_med_max\": [%.1f, %.1f, %.1f], \"xcc_not_blockIdx_mod_8\": %d, "
           "\"by_xcc\": [",
           label, nwg, (t1max - t0min) * 0.01, (t0max - t0min) * 0.01, (t1max - t1min) * 0.01, s[0], s[nwg / 2],
           s[nwg - 1], bad_rr);
    bool first = true;
    for (int x = 0; x < 16; ++x) {
        if (xn[x] == 0) continue;
        printf("%s{\"xcc\": %d, \"wgs\": %.0f, \"mean_us\": %.1f, \"min_us\": %.1f, \"max_us\": %.1f}", first ? "" : ", ",
               x, xn[x], xs[x] / xn[x], xmin[x], xmax[x]);
        first = false;
    }
    printf("], \"by_se_in_xcc\": [");
    first = true;
    for (int x = 0; x < 8; ++x) {
        if (se_n[x] == 0) continue;
        printf("%s{\"se\": %d, \"wgs\": %.0f, \"mean_us\": %.1f}", first ? "" : ", ", x, se_n[x], se_s[x] / se_n[x]);
        first = false;
    }
    printf("]}\n");
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    g_reps = argc > 2 ? atoi(argv[2]) : 10;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t nmax = 1ull << lg;
    uint32_t *a, *b, *sink;
    CK(hipMalloc(&a, nmax * 4));
    CK(hipMalloc(&b, nmax * 4));
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipMemset(a, 1, nmax * 4));
    CK(hipMemset(b, 2, nmax * 4));
    unsigned long long *rec;
    const int max_wg = cus * 32;
    CK(hipMalloc(&rec, (size_t)max_wg * 4 * 8));
    if (argc > 3 && argv[3][0] == 'c') {
        // `c2`: the C2 pass's write-stream floor (2^26 keys, 4096-key tiles, 16 regions, 1024 chunks) beside a
        // plain one-chunk-per-workgroup copy of the same buffers, loads non-temporal, stores both policies
        const uint64_t n = 1ull << 26;
        constexpr int TH = 256, Q = 4;
        constexpr uint32_t T = TH * Q * 4;
        const uint64_t tiles = n / T;
        const uint32_t chunks = 1024, tpc = (uint32_t)(tiles / chunks);
        const u32x4 *A = (const u32x4 *)a;
        double ms = timeit([&] { runs_rg<TH, Q, 16, true, true><<<chunks, TH>>>(A, b, n, tpc); });
        line("c2_runs256_16regions", "chunk", TH, Q, 4, 1, 1, 8.0 * n, ms);
        ms = timeit([&] { runs_rg<TH, Q, 16, true, false><<<chunks, TH>>>(A, b, n, tpc); });
        line("c2_runs256_16regions", "chunk", TH, Q, 4, 1, 0, 8.0 * n, ms);
        ms = timeit([&] { runs_rg<TH, Q, 16, false, false><<<chunks, TH>>>(A, b, n, tpc); });
        line("c2_runs256_16regions", "chunk", TH, Q, 4, 0, 0, 8.0 * n, ms);
        const uint64_t c4 = n / 4 / chunks;
        ms = timeit([&] { copy_chunk<TH, Q, true, true><<<chunks, TH>>>(A, (u32x4 *)b, c4, nullptr); });
        line("c2_copy", "chunk", TH, Q, 4, 1, 1, 8.0 * n, ms);
        ms = timeit([&] { copy_chunk<TH, Q, true, false><<<chunks, TH>>>(A, (u32x4 *)b, c4, nullptr); });
        line("c2_copy", "chunk", TH, Q, 4, 1, 0, 8.0 * n, ms);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'p') {
        // `pairs`: the pairs pass's write-stream floor (8192-pair tiles, runs of 32 pairs in both arrays,
        // one chunk per CU) beside the keys pass's (runs64), 2^lg pairs: four 4 x 2^lg-B buffers
        uint32_t *a2, *b2;
        CK(hipMalloc(&a2, nmax * 4 + (4u << 20)));
        CK(hipMalloc(&b2, nmax * 4 + (4u << 20)));
        CK(hipMemset(a2, 3, nmax * 4 + (4u << 20)));
        const uint64_t n = nmax;
        printf("{\"kind\": \"buffers\", \"a\": \"%p\", \"a2\": \"%p\", \"b\": \"%p\", \"b2\": \"%p\"}\n", (void *)a,
               (void *)a2, (void *)b, (void *)b2);
        {
            // the values arrays moved by a few offsets (bytes): does the two-array floor depend on where the
            // second array of each pair sits relative to the first?
            constexpr int TH = 1024, Q = 2;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            for (uint64_t off : {0ull, 1024ull, 4096ull, 65536ull + 256ull, 2097152ull + 4096ull}) {
                const u32x4 *K = (const u32x4 *)a, *V = (const u32x4 *)(a2 + off / 4);
                double ms = timeit([&] { runs_pairs<TH, Q, true, true><<<g, TH>>>(K, V, b, b2 + off / 4, n, tpc); });
                printf("{\"kind\": \"runs32_pairs_off\", \"offset\": %llu, \"ms\": %.4f, \"TBs\": %.3f}\n",
                       (unsigned long long)off, ms, 16.0 * n / ms / 1e9);
            }
        }
        {
            constexpr int TH = 1024, Q = 2;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            const u32x4 *K = (const u32x4 *)a, *V = (const u32x4 *)a2;
            double ms = timeit([&] { runs_pairs<TH, Q, false, true><<<g, TH>>>(K, V, b, b2, n, tpc); });
            line("runs32_pairs", "chunk", TH, Q, 1, 0, 1, 16.0 * n, ms);
            ms = timeit([&] { runs_pairs<TH, Q, true, true><<<g, TH>>>(K, V, b, b2, n, tpc); });
            line("runs32_pairs", "chunk", TH, Q, 1, 1, 1, 16.0 * n, ms);
            ms = timeit([&] { runs_pairs<TH, Q, false, false><<<g, TH>>>(K, V, b, b2, n, tpc); });
            line("runs32_pairs", "chunk", TH, Q, 1, 0, 0, 16.0 * n, ms);
        }
        {
            constexpr int TH = 1024, Q = 4;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            double ms = timeit([&] { runs<TH, Q, true, true><<<g, TH>>>((const u32x4 *)a, b, n, tpc); });
            line("runs64", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
        }
        {
            constexpr int TH = 1024, Q = 4;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            const u32x4 *A4 = (const u32x4 *)a;
            double ms = timeit([&] { runs_split<TH, Q, true, false><<<g, TH>>>(A4, b, b2, n, tpc); });
            line("runs64_splitread", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
            ms = timeit([&] { runs_split<TH, Q, false, true><<<g, TH>>>(A4, b, b2, n, tpc); });
            line("runs64_splitwrite", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
            ms = timeit([&] { runs_split<TH, Q, true, true><<<g, TH>>>(A4, b, b2, n, tpc); });
            line("runs64_splitboth", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
            ms = timeit([&] { runs_split<TH, Q, false, false><<<g, TH>>>(A4, b, b2, n, tpc); });
            line("runs64_split_none", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
        }
        {
            // keys in 8192-key tiles: runs of 32 keys (128 B), as the pairs stream writes per array
            constexpr int TH = 1024, Q = 2;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            double ms = timeit([&] { runs<TH, Q, true, true><<<g, TH>>>((const u32x4 *)a, b, n, tpc); });
            line("runs32", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
        }
        {
            // pairs in 16384-pair tiles: runs of 64 pairs (256 B) per array
            constexpr int TH = 1024, Q = 4;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            const u32x4 *K = (const u32x4 *)a, *V = (const u32x4 *)a2;
            double ms = timeit([&] { runs_pairs<TH, Q, true, true><<<g, TH>>>(K, V, b, b2, n, tpc); });
            line("runs64_pairs", "chunk", TH, Q, 1, 1, 1, 16.0 * n, ms);
        }
        return 0;
    }
    for (int sz : {lg, 26}) {
        const uint64_t n = 1ull << sz, n4 = n / 4;
        const char *lbl = sz == lg ? "stride_big" : "stride_256MiB";
        const u32x4 *A = (const u32x4 *)a;
        u32x4 *B = (u32x4 *)b;
        stride_set<256, 4, false, false>(A, B, n4, cus, lbl);
        stride_set<256, 4, true, true>(A, B, n4, cus, lbl);
        stride_set<256, 4, true, false>(A, B, n4, cus, lbl);
        stride_set<256, 4, false, true>(A, B, n4, cus, lbl);
        stride_set<1024, 4, false, false>(A, B, n4, cus, lbl);
        stride_set<1024, 4, true, true>(A, B, n4, cus, lbl);
        stride_set<256, 8, true, true>(A, B, n4, cus, lbl);
        stride_set<256, 1, false, false>(A, B, n4, cus, lbl);
        stride_set<256, 1, true, true>(A, B, n4, cus, lbl);
        stride_set<1024, 16, true, true>(A, B, n4, cus, lbl);
        if (sz != lg) continue;
        for (int g : {1, 4, 8, 16}) {
            double ms = timeit([&] { read_only<256, 4, true><<<cus * g, 256>>>(A, sink, n4); });
            line("read", "stride_big", 256, 4, g, 1, 0, 16.0 * n4, ms);
            ms = timeit([&] { read_only<256, 4, false><<<cus * g, 256>>>(A, sink, n4); });
            line("read", "stride_big", 256, 4, g, 0, 0, 16.0 * n4, ms);
            ms = timeit([&] { write_only<256, 4, true><<<cus * g, 256>>>(B, n4); });
            line("write", "stride_big", 256, 4, g, 0, 1, 16.0 * n4, ms);
            ms = timeit([&] { write_only<256, 4, false><<<cus * g, 256>>>(B, n4); });
            line("write", "stride_big", 256, 4, g, 0, 0, 16.0 * n4, ms);
        }
        // one chunk per workgroup (the sort's layout): 1024 x 16 per CU (the line kernels' shape), and
        // 256 x 4 at 4 and 16 workgroups per CU
        {
            const uint64_t chunk4 = n4 / cus;
            double ms = timeit([&] { copy_chunk<1024, 16, true, true><<<cus, 1024>>>(A, B, chunk4, nullptr); });
            line("copy", "chunk", 1024, 16, 1, 1, 1, 32.0 * chunk4 * cus, ms);
            ms = timeit([&] { copy_chunk<1024, 4, false, true><<<cus, 1024>>>(A, B, chunk4, nullptr); });
            line("copy", "chunk", 1024, 4, 1, 0, 1, 32.0 * chunk4 * cus, ms);
            for (int g : {4, 16}) {
                const uint64_t c4 = n4 / (cus * g);
                ms = timeit([&] { copy_chunk<256, 4, true, true><<<cus * g, 256>>>(A, B, c4, nullptr); });
                line("copy", "chunk", 256, 4, g, 1, 1, 32.0 * c4 * cus * g, ms);
            }
            // per-workgroup rates: 3 launches each, every record printed
            std::vector<unsigned long long> h((size_t)max_wg * 4);
            for (int rep = 0; rep < 3; ++rep) {
                copy_chunk<1024, 16, true, true><<<cus, 1024>>>(A, B, chunk4, rec);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h.data(), rec, (size_t)cus * 32, hipMemcpyDeviceToHost));
                chunk_rates("chunk 1024x16 1/CU", h, cus);
            }
            for (int rep = 0; rep < 2; ++rep) {
                const uint64_t c4 = n4 / (cus * 4);
                copy_chunk<256, 4, true, true><<<cus * 4, 256>>>(A, B, c4, rec);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h.data(), rec, (size_t)cus * 4 * 32, hipMemcpyDeviceToHost));
                chunk_rates("chunk 256x4 4/CU", h, cus * 4);
            }
            // the raw records of one 1-per-CU launch, for offline correlation (wg, us, hw_id, xcc)
            copy_chunk<1024, 16, true, true><<<cus, 1024>>>(A, B, chunk4, rec);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), rec, (size_t)cus * 32, hipMemcpyDeviceToHost));
            printf("{\"kind\": \"chunk_records\", \"mode\": \"chunk 1024x16 1/CU\", \"records\": [");
            for (int i = 0; i < cus; ++i)
                printf("%s[%d, %.2f, %.2f, %llu, %llu]", i ? ", " : "", i, (h[4 * i] - h[0]) * 0.01,
                       (h[4 * i + 1] - h[4 * i]) * 0.01, h[4 * i + 2], h[4 * i + 3]);
            printf("]}\n");
        }
        // the keys pass's write stream (16384-key tiles, runs of 64 keys), one chunk per CU
        {
            constexpr int TH = 1024, Q = 4;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            double ms = timeit([&] { runs<TH, Q, false, false><<<g, TH>>>(A, b, n, tpc); });
            line("runs64", "chunk", TH, Q, 1, 0, 0, 8.0 * n, ms);
            ms = timeit([&] { runs<TH, Q, true, true><<<g, TH>>>(A, b, n, tpc); });
            line("runs64", "chunk", TH, Q, 1, 1, 1, 8.0 * n, ms);
            ms = timeit([&] { runs<TH, Q, false, true><<<g, TH>>>(A, b, n, tpc); });
            line("runs64", "chunk", TH, Q, 1, 0, 1, 8.0 * n, ms);
        }
    }
    return 0;
}
