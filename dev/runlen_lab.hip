// Backs DESIGN §3 "Whole-line writes" and §8: the HBM floor of the scatter write stream vs run length and offset (128-B runs 1.67 ms per 2^30 keys; pairs: 128-B runs 2.90 ms, 64-B offset 3.74 ms).
// runlen_lab.hip -- development harness: HBM cost of an LSD-scatter-shaped write stream as a
// function of the run length. A persistent grid walks chunks of 16384-key tiles; each tile is read
// with coalesced 16-B loads and written as T/L runs of L keys (16-B stores, whole aligned lines),
// run r of every tile continuing region r where the same chunk's previous tile stopped -- the
// address stream of a pass whose digit runs are L keys long. Same bytes for every L.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/runlen_lab.hip -o dev/runlen_lab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int THREADS, int QPT>
__global__ __launch_bounds__(THREADS) void runs(const u32x4 *__restrict__ in, uint32_t *__restrict__ out, uint64_t n,
                                                 uint32_t L, uint32_t tpc, uint32_t skew) {
    constexpr uint32_t T = THREADS * QPT * 4;
    const uint32_t R = T / L;
    const uint64_t region = n / R - 32;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 v[QPT];
#pragma unroll
        for (int j = 0; j < QPT; ++j) v[j] = in[tb / 4 + threadIdx.x + j * THREADS];
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const uint32_t i = (threadIdx.x + j * THREADS) * 4;
            const uint32_t r = i / L;
            // skew: every region (and so every run) starts `skew` keys past a 128-B boundary
            const uint64_t pos = r * region + skew + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            *reinterpret_cast<u32x4 *>(out + pos) = v[j];
        }
    }
}

// the same for key + value pairs: two input arrays read, two output arrays written with the same
// runs (a pairs pass: 8192-pair tiles, 256 regions -> runs of 32 pairs = 128 B per array)
template <int THREADS, int QPT>
__global__ __launch_bounds__(THREADS) void runs_pairs(const u32x4 *__restrict__ in, const u32x4 *__restrict__ vin,
                                                       uint32_t *__restrict__ out, uint32_t *__restrict__ vout,
                                                       uint64_t n, uint32_t L, uint32_t tpc, uint32_t skew) {
    constexpr uint32_t T = THREADS * QPT * 4;
    const uint32_t R = T / L;
    const uint64_t region = n / R - 32;
    const uint64_t cbeg = (uint64_t)blockIdx.x * tpc * T;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb + T > n) break;
        u32x4 v[QPT], w[QPT];
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            v[j] = in[tb / 4 + threadIdx.x + j * THREADS];
            w[j] = vin[tb / 4 + threadIdx.x + j * THREADS];
        }
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const uint32_t i = (threadIdx.x + j * THREADS) * 4;
            const uint32_t r = i / L;
            const uint64_t pos = r * region + skew + (uint64_t)blockIdx.x * tpc * L + (uint64_t)tile * L + (i % L);
            __builtin_nontemporal_store(v[j], reinterpret_cast<u32x4 *>(out + pos));
            __builtin_nontemporal_store(w[j], reinterpret_cast<u32x4 *>(vout + pos));
        }
    }
}

template <int THREADS, int QPT>
__global__ __launch_bounds__(THREADS) void copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, uint64_t n4) {
    for (uint64_t b = (uint64_t)blockIdx.x * THREADS * QPT; b < n4; b += (uint64_t)gridDim.x * THREADS * QPT) {
        u32x4 v[QPT];
#pragma unroll
        for (int j = 0; j < QPT; ++j) v[j] = in[b + threadIdx.x + j * THREADS];
#pragma unroll
        for (int j = 0; j < QPT; ++j) out[b + threadIdx.x + j * THREADS] = v[j];
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
        printf("%-48s %8.3f ms %8.1f GB/s\n", name, ms, 8.0 * n / ms / 1e6);
        fflush(stdout);
    };
    char nm[128];
    for (int g : {1, 2, 4}) {
        snprintf(nm, sizeof nm, "copy 256x4q grid=%d/CU", g);
        timeit(nm, [&] { copy<256, 4><<<cus * g, 256>>>((const u32x4 *)a, (u32x4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "copy 1024x4q grid=%d/CU", g);
        timeit(nm, [&] { copy<1024, 4><<<cus * g, 1024>>>((const u32x4 *)a, (u32x4 *)b, n / 4); });
    }
    // 256 regions (a k = 8 pass) from 16384-, 24576- and 32768-key tiles: runs of 64, 96, 128 keys
    auto regions256 = [&](auto qtag) {
        constexpr int Q = decltype(qtag)::value;
        constexpr int TH = 1024;
        constexpr uint32_t T = TH * Q * 4;
        const uint64_t tiles = n / T;
        const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
        const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
        snprintf(nm, sizeof nm, "256 regions, %5u-key tiles: runs of %u keys", T, T / 256);
        timeit(nm, [&] { runs<TH, Q><<<g, TH>>>((const u32x4 *)a, b, n, T / 256, tpc, 0); });
    };
    {
        // pairs: 2^lg pairs = two arrays each way (16 B per pair); value buffers of the same size
        uint32_t *va, *vb;
        CK(hipMalloc(&va, n * 4));
        CK(hipMalloc(&vb, n * 4));
        CK(hipMemset(va, 3, n * 4));
        for (uint32_t skew : {0u, 16u}) {
            constexpr int TH = 512, Q = 4;  // 8192-pair tiles
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            snprintf(nm, sizeof nm, "pairs, 8192-pair tiles, runs of 32, skew %u (x2 bytes)", skew);
            timeit(nm, [&] { runs_pairs<TH, Q><<<g, TH>>>((const u32x4 *)a, (const u32x4 *)va, b, vb, n, T / 256, tpc, skew); });
        }
        {
            constexpr int TH = 1024, Q = 4;  // 16384-pair tiles: runs of 64 pairs
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t tpc = (uint32_t)((tiles + cus - 1) / cus);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            timeit("pairs, 16384-pair tiles, runs of 64 (x2 bytes)", [&] { runs_pairs<TH, Q><<<g, TH>>>((const u32x4 *)a, (const u32x4 *)va, b, vb, n, T / 256, tpc, 0); });
        }
        CK(hipFree(va));
        CK(hipFree(vb));
    }
    regions256(std::integral_constant<int, 4>{});
    regions256(std::integral_constant<int, 6>{});
    regions256(std::integral_constant<int, 8>{});
    for (uint32_t L : {32u, 64u, 128u}) {
        for (uint32_t skew : {0u, 16u, 8u, 4u}) {
            constexpr int TH = 1024, Q = 4;
            constexpr uint32_t T = TH * Q * 4;
            const uint64_t tiles = n / T;
            const uint32_t chunks = cus;
            const uint32_t tpc = (uint32_t)((tiles + chunks - 1) / chunks);
            const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
            snprintf(nm, sizeof nm, "runs 1024x16 L=%-4u (%4u B) skew=%-2u keys", L, L * 4, skew);
            timeit(nm, [&] { runs<TH, Q><<<g, TH>>>((const u32x4 *)a, b, n, L, tpc, skew); });
        }
    }
    return 0;
}
