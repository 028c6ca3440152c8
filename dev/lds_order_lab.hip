// Backs DESIGN §3 "Ranking": gfx950 serves same-address ds_add_rtn lanes in lane order (the kRankAtomic premise).
// lds_order_lab.hip -- does a wave64 ds_add_rtn_u32 whose lanes hit the same LDS address
// return values in ascending lane order (lane i gets old + #lower lanes with that address)?
// If it always does, the per-wave digit rank of a key is one returning LDS atomic and the
// peer-match ballots are unnecessary. Counts violations over many random digit patterns,
// several digit ranges, counter layouts and occupancies.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/lds_order_lab.hip -o dev/lds_order_lab
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

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// Each wave owns R counters (layout: w*R + d, or d*W + w when INTERLEAVE). ITER rounds; per round
// every lane picks a digit (hash, masked to R-1; mode 1 = only 3 distinct digits; mode 2 =
// all lanes one digit), does ret = atomicAdd(&cnt[...], inc) and checks ret against the
// lane-ordered expectation computed from ballots. inc = 1 or lane-dependent (1 + (lane & 3)).
template <int THREADS, bool INTERLEAVE, int RMAX>
__global__ __launch_bounds__(THREADS) void order_test(uint32_t R, int mode, int var_inc, int iters, uint32_t seed,
                                                      unsigned long long *bad, unsigned long long *total) {
    constexpr int W = THREADS / 64;
    __shared__ uint32_t cnt[W * RMAX];
    if (R > RMAX) return;
    const uint32_t t = threadIdx.x, w = t / 64, lane = t % 64;
    for (uint32_t i = t; i < W * R; i += THREADS) cnt[i] = 0;
    __syncthreads();
    unsigned long long nbad = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t h = hash32(seed ^ (blockIdx.x * 0x9E3779B9u) ^ (it * 0x85EBCA6Bu) ^ (t * 0xC2B2AE35u));
        uint32_t d = h & (R - 1);
        if (mode == 1) d = (h % 3u) & (R - 1);
        if (mode == 2) d = (seed + it) & (R - 1);
        const uint32_t inc = var_inc ? 1u + (lane & 3u) : 1u;
        const uint32_t idx = INTERLEAVE ? d * W + w : w * R + d;
        // expected: counter value before this instruction + sum of inc over lower lanes with d
        const uint32_t before = cnt[idx];
        uint32_t below = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t dl = __shfl(d, l);
            const uint32_t il = __shfl(inc, l);
            if ((uint32_t)l < lane && dl == d) below += il;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t ret = atomicAdd(&cnt[idx], inc);
        if (ret != before + below) ++nbad;
        __builtin_amdgcn_wave_barrier();
    }
    atomicAdd(bad, nbad);
    atomicAdd(total, (unsigned long long)iters);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long *d;
    CK(hipMalloc(&d, 16));
    unsigned long long h[2];
    auto run = [&](const char *name, auto kern, int threads, uint32_t R, int mode, int var_inc, int bpc) {
        CK(hipMemset(d, 0, 16));
        kern<<<cus * bpc, threads>>>(R, mode, var_inc, iters, 0x1234u + R * 7 + mode, d, d + 1);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("%-12s threads=%4d R=%4u mode=%d var_inc=%d bpc=%d  lane-ops=%llu  violations=%llu\n", name, threads, R,
               mode, var_inc, bpc, h[1], h[0]);
        fflush(stdout);
    };
    for (uint32_t R : {1u, 2u, 16u, 256u, 4096u}) {
        for (int mode : {0, 1, 2}) {
            for (int vi : {0, 1}) {
                run("w*R+d", order_test<512, false, 4096>, 512, R, mode, vi, 2);
                if (R <= 512) run("d*W+w", order_test<512, true, 512>, 512, R, mode, vi, 2);
            }
        }
    }
    run("w*R+d", order_test<256, false, 256>, 256, 256, 0, 0, 4);
    run("w*R+d", order_test<1024, false, 256>, 1024, 256, 0, 0, 1);
    return 0;
}
