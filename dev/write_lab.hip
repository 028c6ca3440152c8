// write_lab.hip -- development harness: HBM ceilings for the sort's access patterns.
//   copy kernels (dword / dwordx4, several grid shapes), and a synthetic "run scatter" that
//   reads tiles coalesced and writes each tile as R runs of L = T/R keys to R regions, the
//   same address stream an LSD scatter pass produces for uniform keys, with no ranking work.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/write_lab.hip -o dev/write_lab
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

template <int U>
__global__ __launch_bounds__(256) void copy_x4(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n4) ? in[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) out[i + u * 256] = v[u];
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void copy_x4_nt(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, uint64_t n4) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n4) ? __builtin_nontemporal_load(&in[i + u * 256]) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) __builtin_nontemporal_store(v[u], &out[i + u * 256]);
    }
}

__global__ __launch_bounds__(256) void read_only(const uint4 *__restrict__ in, uint64_t n4, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
        uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void write_only(uint4 *__restrict__ out, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256)
        out[i] = make_uint4(i, i, i, i);
}

// Synthetic run scatter: chunk c (one workgroup) walks tiles of T = 256*KPT keys; key i of a
// tile goes to region d = i / L at region_base(d, c) + tile*L + (i % L). Reads striped dwords
// (like the sort), writes dwords from "LDS order" (thread t handles positions t + j*256).
template <int KPT>
__global__ __launch_bounds__(256) void run_scatter(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                   uint64_t n, uint32_t R, uint32_t tiles_per_chunk, int use_lds,
                                                   uint32_t skew = 0) {
    constexpr uint32_t T = 256 * KPT;
    __shared__ uint32_t s[T];
    const uint32_t L = T / R;
    const uint64_t region = n / R;              // keys per region
    const uint64_t cbeg = (uint64_t)blockIdx.x * tiles_per_chunk * T;
    const uint64_t per_chunk_region = (uint64_t)tiles_per_chunk * L;
    const uint32_t w = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (uint32_t tile = 0; tile < tiles_per_chunk; ++tile) {
        const uint64_t tb = cbeg + (uint64_t)tile * T;
        if (tb >= n) break;
        uint32_t k[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = in[tb + w * 64 * KPT + j * 64 + lane];
        if (use_lds) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) s[w * 64 * KPT + j * 64 + lane] = k[j];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = s[threadIdx.x + j * 256];
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t i = threadIdx.x + j * 256;
            const uint32_t d = i / L;
            uint64_t pos = d * region + blockIdx.x * per_chunk_region + (uint64_t)tile * L + (i % L);
            pos = (pos + (uint64_t)d * skew) % n;  // skew: runs start off 128-B line boundaries
            out[pos] = k[j];
        }
    }
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = 1ull << lg;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *a, *b, *sink;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, n * 4));
    CK(hipMemset(b, 2, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, double bytes, auto f) {
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
        printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    const uint64_t n4 = n / 4;
    const double cb = 8.0 * n;
    for (int g : {1, 2, 4, 8, 16}) {
        char nm[64];
        snprintf(nm, 64, "copy x4 U=1 grid=%d/CU", g);
        timeit(nm, cb, [&] { copy_x4<1><<<cus * g, 256>>>((const uint4 *)a, (uint4 *)b, n4); });
        snprintf(nm, 64, "copy x4 U=4 grid=%d/CU", g);
        timeit(nm, cb, [&] { copy_x4<4><<<cus * g, 256>>>((const uint4 *)a, (uint4 *)b, n4); });
    }
    timeit("copy x4 U=4 nt grid=8/CU", cb, [&] { copy_x4_nt<4><<<cus * 8, 256>>>((const u32x4 *)a, (u32x4 *)b, n4); });
    timeit("copy x4 U=1 grid=n4/256", cb, [&] { copy_x4<1><<<(unsigned)(n4 / 256), 256>>>((const uint4 *)a, (uint4 *)b, n4); });
    timeit("read only x4 grid=16/CU", 4.0 * n, [&] { read_only<<<cus * 16, 256>>>((const uint4 *)a, n4, sink); });
    timeit("write only x4 grid=16/CU", 4.0 * n, [&] { write_only<<<cus * 16, 256>>>((uint4 *)b, n4); });
    for (uint32_t skew : {0u, 7u, 13u}) {
        for (int kpt : {16, 32, 64}) {
            const uint32_t R = 256, T = 256 * kpt;
            const uint64_t tiles = n / T;
            for (int bpc : {2, 4}) {
                const uint32_t chunks = cus * bpc;
                const uint32_t tpc = (uint32_t)((tiles + chunks - 1) / chunks);
                char nm[96];
                snprintf(nm, 96, "run_scatter T=%u R=256 L=%u skew=%u bpc=%d", T, T / R, skew, bpc);
                const unsigned g = (unsigned)((tiles + tpc - 1) / tpc);
                if (kpt == 16) timeit(nm, cb, [&] { run_scatter<16><<<g, 256>>>(a, b, n, R, tpc, 1, skew); });
                if (kpt == 32) timeit(nm, cb, [&] { run_scatter<32><<<g, 256>>>(a, b, n, R, tpc, 1, skew); });
                if (kpt == 64) timeit(nm, cb, [&] { run_scatter<64><<<g, 256>>>(a, b, n, R, tpc, 1, skew); });
            }
        }
    }
    return 0;
}
