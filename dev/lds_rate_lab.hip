// Backs DESIGN §3 "Ranking": LDS cycles per wave instruction for the ranking access shapes (127 cycles when 64 lanes share a counter).
// lds_rate_lab.hip -- development harness: LDS cost per wave-instruction for the access shapes
// of the scatter kernel's ranking: random-digit ds_add_u32 / ds_add_rtn_u32 / ds_read_b32 /
// ds_write_b32 / ds_read_b64 into per-wave 256-entry counter arrays, 1024-thread workgroups,
// one per CU. Prints cycles per wave-instruction (s_memtime) and chip time.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/lds_rate_lab.hip -o dev/lds_rate_lab
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

// OP: 0 ds_add_u32, 1 ds_add_rtn_u32, 2 ds_read_b32, 3 ds_write_b32, 4 ds_read_b64 (uint2 array)
// RANGE: distinct digits per wave (256 random, 16, 1 = all lanes same address)
template <int OP>
__global__ __launch_bounds__(1024) void lds_rate(uint32_t range, int iters, uint32_t *sink, unsigned long long *cyc) {
    __shared__ uint32_t cnt[16 * 512];
    const uint32_t t = threadIdx.x, w = t / 64;
    for (uint32_t i = t; i < 16 * 512; i += 1024) cnt[i] = 0;
    __syncthreads();
    uint32_t d[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) d[j] = hash32(t * 16 + j + blockIdx.x * 7919) % range;
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            asm volatile("" : "+v"(d[j]));
            if constexpr (OP == 0) atomicAdd(&cnt[w * 256 + d[j]], 1u);
            if constexpr (OP == 1) acc += atomicAdd(&cnt[w * 256 + d[j]], 1u);
            if constexpr (OP == 2) acc += cnt[w * 256 + d[j]];
            if constexpr (OP == 3) cnt[w * 256 + d[j]] = acc + j;
            if constexpr (OP == 4) {
                const uint2 v = reinterpret_cast<const uint2 *>(cnt)[w * 256 + d[j]];
                acc += v.x ^ v.y;
            }
        }
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (acc == 0x12345u) sink[0] = acc;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *sink;
    unsigned long long *cyc;
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&cyc, cus * 8));
    unsigned long long *h = (unsigned long long *)malloc(cus * 8);
    const char *names[5] = {"ds_add_u32", "ds_add_rtn_u32", "ds_read_b32", "ds_write_b32", "ds_read_b64"};
    auto run = [&](int op, auto kern, uint32_t range) {
        kern<<<cus, 1024>>>(range, iters, sink, cyc);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, cyc, cus * 8, hipMemcpyDeviceToHost));
        double avg = 0;
        for (int i = 0; i < cus; ++i) avg += h[i];
        avg /= cus;
        // 16 waves x 16 instructions x iters per CU
        printf("%-16s range=%4u  %8.2f cycles per wave-instruction (CU-wide)\n", names[op], range,
               avg / (16.0 * 16.0 * iters));
        fflush(stdout);
    };
    for (uint32_t range : {256u, 64u, 16u, 1u}) {
        run(0, lds_rate<0>, range);
        run(1, lds_rate<1>, range);
        run(2, lds_rate<2>, range);
        run(3, lds_rate<3>, range);
        run(4, lds_rate<4>, range);
    }
    return 0;
}
