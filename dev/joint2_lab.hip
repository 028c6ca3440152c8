// Backs DESIGN §8 "Histograms": two 8-bit joint tables in one key read are LDS-bound (0.95 ms uniform, 6.8 ms Zipf).
// joint2_lab.hip -- development harness (not part of the library): can pass 0's key read count two
// joint tables at once? Times, over 2^30 keys in 256 chunks (one 1024-thread workgroup each):
//   A  the library's layout: (digit 0, digit 1) pairs in 16-bit LDS counters, spill at 2^15
//   B  (digit 0, digit 1) and (digit 2, digit 3) pairs in two 8-bit LDS tables, spill at 2^7
//      (what a pass-3 digit-group / cut plan would need without pass 2's joint count)
// on uniform keys and on Zipf keys in input order (pass 0's input).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cuda.radixsort_amd/csrc dev/joint2_lab.hip -o dev/joint2_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include "rsort_internal.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(1024) void joint_lab(const uint32_t *keys, uint64_t n, uint32_t *J1, uint32_t *J2, uint32_t *table) {
    constexpr uint32_t R = 256;
    // MODE 0: 16-bit table, rows of 129 words; MODE 1: two 8-bit tables, rows of 65 words
    constexpr uint32_t RS = MODE == 0 ? R / 2 + 1 : R / 4 + 1;
    constexpr uint32_t TW = R * RS;
    __shared__ uint32_t s_t[MODE == 0 ? TW + R : 2 * TW + R];
    uint32_t *s_sp = s_t + (MODE == 0 ? TW : 2 * TW);
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < (MODE == 0 ? TW + R : 2 * TW + R); i += 1024) s_t[i] = 0;
    __syncthreads();
    auto add16 = [&](uint32_t d, uint32_t e) {
        const uint32_t wi = d * RS + (e >> 1), sh = (e & 1u) << 4;
        const uint32_t before = (atomicAdd(&s_t[wi], 1u << sh) >> sh) & 0xFFFFu;
        if (before == 0x7FFFu) {
            atomicSub(&s_t[wi], 0x8000u << sh);
            atomicAdd(&s_sp[d], 0x8000u);
            atomicAdd(&J1[e * R + d], 0x8000u);
        }
    };
    auto add8 = [&](uint32_t *tb, uint32_t *J, uint32_t d, uint32_t e, bool sp) {
        const uint32_t wi = d * RS + (e >> 2), sh = (e & 3u) << 3;
        const uint32_t before = (atomicAdd(&tb[wi], 1u << sh) >> sh) & 0xFFu;
        if (before == 0x7Fu) {
            atomicSub(&tb[wi], 0x80u << sh);
            if (sp) atomicAdd(&s_sp[d], 0x80u);
            atomicAdd(&J[e * R + d], 0x80u);
        }
    };
    auto add = [&](uint32_t x) {
        if constexpr (MODE == 0) {
            add16(x & 255u, (x >> 8) & 255u);
        } else {
            add8(s_t, J1, x & 255u, (x >> 8) & 255u, true);
            add8(s_t + TW, J2, (x >> 16) & 255u, x >> 24, false);
        }
    };
    const uint64_t cb = (uint64_t)blockIdx.x * (n / gridDim.x), ce = cb + n / gridDim.x;
    const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + cb);
    const uint32_t nvec = (uint32_t)((ce - cb) / 4);
    for (uint32_t v0 = t; v0 < nvec; v0 += 4096) {
        u32x4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = v0 + u * 1024 < nvec ? __builtin_nontemporal_load(p + v0 + u * 1024) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (v0 + u * 1024 < nvec) {
                add(q[u].x);
                add(q[u].y);
                add(q[u].z);
                add(q[u].w);
            }
    }
    __syncthreads();
    for (uint32_t d = t; d < R; d += 1024) {
        uint32_t s = s_sp[d];
        for (uint32_t j = 0; j < RS - 1; ++j) {
            const uint32_t x = s_t[d * RS + j];
            s += MODE == 0 ? (x & 0xFFFFu) + (x >> 16) : (x & 0xFFu) + ((x >> 8) & 0xFFu) + ((x >> 16) & 0xFFu) + (x >> 24);
        }
        table[d * gridDim.x + blockIdx.x] = s;
    }
    for (uint32_t item = t; item < R * R; item += 1024) {
        const uint32_t e = item / R, d = item % R;
        if constexpr (MODE == 0) {
            const uint32_t v = (s_t[d * RS + (e >> 1)] >> ((e & 1u) << 4)) & 0xFFFFu;
            if (v) atomicAdd(&J1[item], v);
        } else {
            const uint32_t v1 = (s_t[d * RS + (e >> 2)] >> ((e & 3u) << 3)) & 0xFFu;
            if (v1) atomicAdd(&J1[item], v1);
            const uint32_t v2 = (s_t[TW + d * RS + (e >> 2)] >> ((e & 3u) << 3)) & 0xFFu;
            if (v2) atomicAdd(&J2[item], v2);
        }
    }
}

int main(int argc, char **argv) {
    const uint64_t n = 1ull << 30;
    uint32_t *keys, *J1, *J2, *table;
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&J1, 65536 * 4));
    CK(hipMalloc(&J2, 65536 * 4));
    CK(hipMalloc(&table, 65536 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int dist = 0; dist < 2; ++dist) {
        if (dist == 0) {
            CK(rsort::launch_gen_uniform(keys, n, 0x5EED, 0));
        } else {
            const int ranks = 1 << 20;
            std::vector<double> cum(ranks);
            double acc = 0;
            for (int r = 0; r < ranks; ++r) cum[r] = (acc += 1.0 / (r + 1.0));
            std::vector<uint32_t> cdf(ranks);
            for (int r = 0; r < ranks; ++r) {
                const double tt = floor(cum[r] / acc * 4294967296.0);
                cdf[r] = tt >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)tt;
            }
            cdf[ranks - 1] = 0xFFFFFFFFu;
            uint32_t *d_cdf;
            CK(hipMalloc(&d_cdf, ranks * 4));
            CK(hipMemcpy(d_cdf, cdf.data(), ranks * 4, hipMemcpyHostToDevice));
            CK(rsort::launch_gen_zipf(keys, n, 0x5EED, d_cdf, ranks, 0));
        }
        CK(hipDeviceSynchronize());
        for (int rep = 0; rep < 2; ++rep)
            for (int mode = 0; mode < 2; ++mode) {
                float best = 1e9f;
                for (int it = 0; it < 5; ++it) {
                    CK(hipMemset(J1, 0, 65536 * 4));
                    CK(hipMemset(J2, 0, 65536 * 4));
                    CK(hipEventRecord(e0));
                    if (mode == 0) joint_lab<0><<<256, 1024>>>(keys, n, J1, J2, table);
                    else joint_lab<1><<<256, 1024>>>(keys, n, J1, J2, table);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms < best ? ms : best;
                }
                // check: the joint counts add up to n
                std::vector<uint32_t> h(65536);
                CK(hipMemcpy(h.data(), J1, 65536 * 4, hipMemcpyDeviceToHost));
                unsigned long long s1 = 0;
                for (uint32_t v : h) s1 += v;
                unsigned long long s2 = 0;
                if (mode == 1) {
                    CK(hipMemcpy(h.data(), J2, 65536 * 4, hipMemcpyDeviceToHost));
                    for (uint32_t v : h) s2 += v;
                }
                printf("%-8s %-36s %7.3f ms  sum1=%llu sum2=%llu\n", dist ? "zipf" : "uniform",
                       mode ? "B two 8-bit tables (d0,d1)+(d2,d3)" : "A one 16-bit table (d0,d1)", best, s1, s2);
                fflush(stdout);
            }
    }
    return 0;
}
