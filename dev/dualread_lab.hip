// Backs DESIGN §8 "Histograms": two concurrent readers of one chunk cost two reads (request-rate bound).
// dualread_lab.hip -- development harness: can two workgroups count the same chunk of keys for the
// price of one HBM read? 256 chunks of n/256 keys; each workgroup (1024 threads, one per CU: 128 KB
// of LDS) reads its chunk with non-temporal 16-B loads and adds one LDS atomic per key (a
// histogram-shaped load). Grid 256: one reader per chunk. Grid 512: workgroups 2c and 2c + 1 both
// read chunk c at the same time (the second read may come from the Infinity Cache).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/dualread_lab.hip -o dev/dualread_lab
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

// READERS workgroups per chunk; shift: which byte each reader counts (reader r: byte r)
template <int READERS>
__global__ __launch_bounds__(1024) void count(const u32x4 *__restrict__ keys, uint64_t chunk_q, uint32_t *out) {
    __shared__ uint32_t s_h[32768];  // 128 KB: one workgroup per CU, like the joint histogram
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 32768; i += 1024) s_h[i] = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x / READERS, r = blockIdx.x % READERS;
    const u32x4 *p = keys + (uint64_t)c * chunk_q;
    const uint32_t sh = 8 * r;
    constexpr int U = 4;
    for (uint64_t v0 = t; v0 < chunk_q; v0 += 1024 * U) {
        u32x4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = v0 + u * 1024 < chunk_q ? __builtin_nontemporal_load(p + v0 + u * 1024) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) {
            atomicAdd(&s_h[((q[u].x >> sh) & 255u) * 128 + (t & 127)], 1u);
            atomicAdd(&s_h[((q[u].y >> sh) & 255u) * 128 + (t & 127)], 1u);
            atomicAdd(&s_h[((q[u].z >> sh) & 255u) * 128 + (t & 127)], 1u);
            atomicAdd(&s_h[((q[u].w >> sh) & 255u) * 128 + (t & 127)], 1u);
        }
    }
    __syncthreads();
    if (t < 256) {
        uint32_t s = 0;
        for (int i = 0; i < 128; ++i) s += s_h[t * 128 + i];
        atomicAdd(&out[r * 256 + t], s);
    }
}

__global__ void gen(uint32_t *k, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x5EED;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        k[i] = (uint32_t)((z ^ (z >> 31)) >> 32);
    }
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = 1ull << lg;
    uint32_t *k, *out, *flush;
    CK(hipMalloc(&k, n * 4));
    CK(hipMalloc(&flush, n * 4));
    CK(hipMalloc(&out, 4096 * 4));
    gen<<<4096, 256>>>(k, n);
    gen<<<4096, 256>>>(flush, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t chunk_q = n / 256 / 4;
    auto timeit = [&](const char *name, auto f) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            count<1><<<256, 1024>>>((const u32x4 *)flush, chunk_q, out);  // other data in the caches
            CK(hipEventRecord(e0, 0));
            f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        CK(hipGetLastError());
        printf("%-52s %8.3f ms  %7.1f GB/s of keys\n", name, best, 4.0 * n / best / 1e6);
        fflush(stdout);
    };
    for (int i = 0; i < 2; ++i) {
        timeit("1 reader per chunk (256 workgroups)", [&] { count<1><<<256, 1024>>>((const u32x4 *)k, chunk_q, out); });
        timeit("2 readers per chunk, same time (512 workgroups)", [&] { count<2><<<512, 1024>>>((const u32x4 *)k, chunk_q, out); });
        timeit("3 readers per chunk, same time (768 workgroups)", [&] { count<3><<<768, 1024>>>((const u32x4 *)k, chunk_q, out); });
        timeit("1 reader, twice (two launches)", [&] {
            count<1><<<256, 1024>>>((const u32x4 *)k, chunk_q, out);
            count<1><<<256, 1024>>>((const u32x4 *)k, chunk_q, out);
        });
    }
    return 0;
}
