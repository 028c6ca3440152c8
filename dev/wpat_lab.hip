// wpat_lab.hip -- development harness: does the ORDER in which an LSD scatter's digit runs reach
// HBM matter? Same bytes as dev/runlen_lab.hip (each 16384-key tile read with 16-B loads and
// written as T/L runs of L keys into R = T/L regions), three address orders:
//   chunk  (the library's order): workgroup b walks tiles b*tpc .. b*tpc+tpc-1; its runs in region
//          r continue where its previous tile stopped -> 256 x R write streams spread over HBM
//   inter  tiles interleaved: workgroup b walks tiles t*G + b; at any moment the G workgroups
//          write ADJACENT runs of every region (one contiguous front per region)
//   xcd    interleaved with workgroups of one XCD (b % 8 equal) adjacent in the output, so the
//          line shared by two neighbouring runs is written by two CUs behind the same L2
// skew shifts every run by `skew` keys off the 128-B grid (partial first/last lines).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/wpat_lab.hip -o dev/wpat_lab
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum { kChunk = 0, kInter = 1, kXcd = 2 };

template <int THREADS, int QPT, int ORDER, bool NT>
__global__ __launch_bounds__(THREADS) void runs(const u32x4 *__restrict__ in, uint32_t *__restrict__ out, uint64_t n,
                                                 uint32_t L, uint32_t tpc, uint32_t skew) {
    constexpr uint32_t T = THREADS * QPT * 4;
    const uint32_t R = T / L;
    const uint64_t tiles = n / T;
    const uint64_t region = n / R - 64;
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t slot = ORDER == kXcd ? (b % 8) * (G / 8) + b / 8 : b;
    for (uint32_t tile = 0; tile < tpc; ++tile) {
        const uint64_t g = ORDER == kChunk ? (uint64_t)b * tpc + tile : (uint64_t)tile * G + slot;  // output order
        const uint64_t src = ORDER == kChunk ? g : (uint64_t)tile * G + b;                          // input tile
        if (g >= tiles || src >= tiles) break;
        u32x4 v[QPT];
#pragma unroll
        for (int j = 0; j < QPT; ++j)
            v[j] = NT ? __builtin_nontemporal_load(in + src * (T / 4) + threadIdx.x + j * THREADS)
                      : in[src * (T / 4) + threadIdx.x + j * THREADS];
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const uint32_t i = (threadIdx.x + j * THREADS) * 4;
            const uint32_t r = i / L;
            const uint64_t pos = r * region + skew + g * L + (i % L);
            if (NT) __builtin_nontemporal_store(v[j], reinterpret_cast<u32x4 *>(out + pos));
            else *reinterpret_cast<u32x4 *>(out + pos) = v[j];
        }
    }
}

template <int THREADS, int QPT>
__global__ __launch_bounds__(THREADS) void copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, uint64_t n4) {
    for (uint64_t b = (uint64_t)blockIdx.x * THREADS * QPT; b < n4; b += (uint64_t)gridDim.x * THREADS * QPT) {
        u32x4 v[QPT];
#pragma unroll
        for (int j = 0; j < QPT; ++j) v[j] = __builtin_nontemporal_load(in + b + threadIdx.x + j * THREADS);
#pragma unroll
        for (int j = 0; j < QPT; ++j) __builtin_nontemporal_store(v[j], out + b + threadIdx.x + j * THREADS);
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
        printf("%-56s %8.3f ms %8.1f GB/s\n", name, ms, 8.0 * n / ms / 1e6);
        fflush(stdout);
    };
    char nm[128];
    timeit("copy 1024x4q nt grid=1/CU", [&] { copy<1024, 4><<<cus, 1024>>>((const u32x4 *)a, (u32x4 *)b, n / 4); });
    timeit("copy 1024x4q nt grid=2/CU", [&] { copy<1024, 4><<<cus * 2, 1024>>>((const u32x4 *)a, (u32x4 *)b, n / 4); });
    constexpr int TH = 1024, Q = 4;
    constexpr uint32_t T = TH * Q * 4;
    const uint64_t tiles = n / T;
    const uint32_t G = (uint32_t)cus;
    const uint32_t tpc = (uint32_t)((tiles + G - 1) / G);
    const char *onames[3] = {"chunk", "inter", "xcd"};
    for (uint32_t L : {64u, 256u, 1024u}) {
        for (uint32_t skew : {0u, 16u}) {
            for (int o = 0; o < 3; ++o) {
                for (int nt = 0; nt < 2; ++nt) {
                    snprintf(nm, sizeof nm, "runs %-5s L=%-4u skew=%-2u %s", onames[o], L, skew, nt ? "nt" : "plain");
                    auto go = [&] {
                        const u32x4 *ia = (const u32x4 *)a;
                        if (o == 0 && nt) runs<TH, Q, kChunk, true><<<G, TH>>>(ia, b, n, L, tpc, skew);
                        if (o == 0 && !nt) runs<TH, Q, kChunk, false><<<G, TH>>>(ia, b, n, L, tpc, skew);
                        if (o == 1 && nt) runs<TH, Q, kInter, true><<<G, TH>>>(ia, b, n, L, tpc, skew);
                        if (o == 1 && !nt) runs<TH, Q, kInter, false><<<G, TH>>>(ia, b, n, L, tpc, skew);
                        if (o == 2 && nt) runs<TH, Q, kXcd, true><<<G, TH>>>(ia, b, n, L, tpc, skew);
                        if (o == 2 && !nt) runs<TH, Q, kXcd, false><<<G, TH>>>(ia, b, n, L, tpc, skew);
                    };
                    timeit(nm, go);
                }
            }
        }
    }
    return 0;
}
