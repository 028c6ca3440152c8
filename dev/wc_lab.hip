// Backs rsort_kernels.hip rs_scatter_lines header: partial-line writes cost as much as whole lines (1.7 ms aligned vs 2.8 ms misaligned).
// wc_lab.hip -- development harness: which cache policy / granularity makes the LSD scatter's
// partial-line writes cheap. Synthetic run scatter (as in write_lab.hip): chunk c walks tiles of
// T = THREADS*KPT keys; key i of a tile goes to region d = i / L at
// region_base(d) + chunk*tpc*L + tile*L + i%L (+ d*skew), i.e. R = T/L runs per tile, each run
// continuing where the same chunk's previous tile left it -- the address stream of a real pass.
//
//   LP (load policy)   0 default, 1 nontemporal
//   SP (store policy)  0 default, 1 nontemporal, 2 nontemporal for whole 64-B segments inside
//                      the run and default for the run's partial head/tail segments,
//                      3 = 2 with 128-B lines as the unit
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/wc_lab.hip -o dev/wc_lab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int THREADS, int KPT, int LP, int SP>
__global__ __launch_bounds__(THREADS) void run_scatter(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                       uint64_t n, uint32_t L, uint32_t tpc, uint32_t skew) {
    constexpr uint32_t T = THREADS * KPT;
    __shared__ uint32_t s[T];
    const uint32_t R = T / L;
    const uint64_t region = n / R;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    const uint64_t per_chunk_region = (uint64_t)tpc * L;
    const uint32_t w = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        uint32_t k[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t *p = &in[tb + w * 64 * KPT + j * 64 + lane];
            k[j] = LP ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) s[w * 64 * KPT + j * 64 + lane] = k[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = s[threadIdx.x + j * THREADS];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t i = threadIdx.x + j * THREADS;
            const uint32_t d = i / L;
            const uint64_t rs = d * region + blockIdx.x * per_chunk_region + (uint64_t)tile * L + (uint64_t)d * skew;
            const uint64_t pos = rs + (i % L);
            if (pos >= n) continue;
            uint32_t *q = &out[pos];
            if constexpr (SP == 0) {
                *q = k[j];
            } else if constexpr (SP == 1) {
                __builtin_nontemporal_store(k[j], q);
            } else {
                constexpr uint32_t G = SP == 2 ? 16u : 32u;
                const uint64_t sb = pos & ~(uint64_t)(G - 1);
                const bool whole = sb >= rs && sb + G <= rs + L;
                if (whole) __builtin_nontemporal_store(k[j], q);
                else *q = k[j];
            }
        }
    }
}

// Same address stream, but written like rs_scatter_lines: each lane stores 16 B (4 keys) with
// dwordx4 from a 16-B-aligned LDS quad, Q lanes per region run, W16 = 1: 4 lanes per 64-B line.
template <int THREADS, int KPT>
__global__ __launch_bounds__(THREADS) void run_scatter_x4(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                          uint64_t n, uint32_t L, uint32_t tpc) {
    constexpr uint32_t T = THREADS * KPT;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint32_t s[T];
    const uint32_t R = T / L;
    const uint64_t region = n / R;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    const uint64_t per_chunk_region = (uint64_t)tpc * L;
    const uint32_t w = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        uint32_t k[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = in[tb + w * 64 * KPT + j * 64 + lane];
#pragma unroll
        for (int j = 0; j < KPT; ++j) s[w * 64 * KPT + j * 64 + lane] = k[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT / 4; ++j) {
            const uint32_t i = (threadIdx.x + j * THREADS) * 4;  // quad start
            const uint32_t d = i / L;
            const uint64_t pos = d * region + blockIdx.x * per_chunk_region + (uint64_t)tile * L + (i % L);
            const u32x4 v = *reinterpret_cast<const u32x4 *>(&s[i]);
            if (pos + 4 <= n) *reinterpret_cast<u32x4 *>(out + pos) = v;
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = 1ull << lg;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 1, n * 4));
    CK(hipMemset(b, 2, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto f) {
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        const int reps = 10;
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-60s %8.3f ms %8.1f GB/s\n", name, ms, 8.0 * n / ms / 1e6);
        fflush(stdout);
    };
#define RUN(TH, KP, LPv, SPv, bpc)                                                                       \
    do {                                                                                                 \
        constexpr uint32_t T = TH * KP;                                                                  \
        const uint64_t tiles = n / T;                                                                    \
        const uint32_t chunks = cus * (bpc);                                                             \
        const uint32_t tpc = (uint32_t)((tiles + chunks - 1) / chunks);                                  \
        const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);                                          \
        char nm[128];                                                                                    \
        snprintf(nm, sizeof nm, "%4dx%-2d L=%-3u skew=%-2u LP=%d SP=%d bpc=%d", TH, KP, L, skew, LPv, SPv, \
                 bpc);                                                                                   \
        timeit(nm, [&] { run_scatter<TH, KP, LPv, SPv><<<g, TH>>>(a, b, n, L, tpc, skew); });            \
    } while (0)
    const uint32_t L = 64;
    for (uint32_t skew : {0u, 4u, 8u, 16u, 7u}) {
        RUN(512, 32, 0, 0, 2);
        if (skew == 0 || skew == 7) {
            RUN(512, 32, 1, 0, 2);
            RUN(512, 32, 0, 1, 2);
            RUN(512, 32, 1, 1, 2);
            RUN(512, 32, 0, 2, 2);
            RUN(512, 32, 1, 2, 2);
            RUN(512, 32, 1, 3, 2);
        }
    }
    {
        const uint32_t skew = 0;
        for (uint32_t L : {64u, 16u, 32u}) {
            for (int bpc : {1, 2}) {
                constexpr int TH = 1024, KP = 16;
                constexpr uint32_t T = TH * KP;
                const uint64_t tiles = n / T;
                const uint32_t chunks = cus * bpc;
                const uint32_t tpc = (uint32_t)((tiles + chunks - 1) / chunks);
                const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
                char nm[128];
                snprintf(nm, sizeof nm, "x4 1024x16 L=%-3u aligned bpc=%d", L, bpc);
                timeit(nm, [&] { run_scatter_x4<TH, KP><<<g, TH>>>(a, b, n, L, tpc); });
                (void)skew;
            }
        }
    }
    {
        // longer runs: 1024 x 32 (T = 32768, L = 128) at one workgroup per CU
        const uint32_t L = 128;
        for (uint32_t skew : {0u, 7u}) {
            RUN(1024, 32, 0, 0, 1);
            RUN(1024, 32, 1, 2, 1);
        }
    }
    return 0;
}
