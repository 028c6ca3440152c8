// dev/lab_hooks.hpp -- the lab side of cuda.radixsort_amd/csrc/rsort_hooks.hpp: included by it when a lab build
// passes -DRSORT_LAB_HOOKS='"/root/repo/dev/lab_hooks.hpp"' (dev/build_variant.sh, the dev/*_lab.hip builds).
// It defines every hook the library's kernels call, with these switches (each -D on the hipcc line):
//   RSORT_DEFER_KEYS_CL / RSORT_DEFER_KEYS_PLAIN / RSORT_DEFER_PAIRS   deferred-ranking batch sizes (2 / 0 / 4)
//   RSORT_NXR                 next-digit counter replicas (8)
//   RSORT_LINES_MINW_SMALL    minimum waves per SIMD of the 256-thread line kernels (1)
//   RSORT_WG_TIMES            every rs_scatter_lines workgroup (the first 2048 of a pass; slot = shift / BITS)
//                             and every joint-count histogram workgroup records its start and end
//                             (s_memrealtime, 100 MHz) and key range, read back with rsort_lab_wg_times
//                             (dev/wgtimes_lab.py); the upper halves of the range words hold where it ran:
//                             HW_ID (hwreg 4: cu 11:8, sh 12, se 15:13) over beg, XCC_ID (hwreg 20) over end
//   RSORT_STAMPS              per-phase s_memtime cycle totals of thread 0 into ScatterArgs::stamps
//                             [workgroup * 8 + phase] (rs_scatter_pairs, dev/pairs_lab.hip)
//   RSORT_LAB_NO_STORES       the scatter kernels' output stores compiled out (the values they would store kept
//                             live): the LDS / VALU floor of a pass (DESIGN §3 "Floors"; the output is garbage)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef RSORT_DEFER_KEYS_CL
#define RSORT_DEFER_KEYS_CL 2
#endif
#ifndef RSORT_DEFER_KEYS_PLAIN
#define RSORT_DEFER_KEYS_PLAIN 0
#endif
#ifndef RSORT_DEFER_PAIRS
#define RSORT_DEFER_PAIRS 4
#endif
#ifndef RSORT_NXR
#define RSORT_NXR 8
#endif
#ifndef RSORT_LINES_MINW_SMALL
#define RSORT_LINES_MINW_SMALL 1
#endif

namespace rsort {
namespace hooks {
constexpr int kDeferKeysCl = RSORT_DEFER_KEYS_CL;
constexpr int kDeferKeysPlain = RSORT_DEFER_KEYS_PLAIN;
constexpr int kDeferPairs = RSORT_DEFER_PAIRS;
constexpr int kNextReplicas = RSORT_NXR;
constexpr int kLinesMinWavesSmall = RSORT_LINES_MINW_SMALL;

typedef uint32_t u32x4h __attribute__((ext_vector_type(4)));
#ifdef RSORT_LAB_NO_STORES
// keep what would be stored live (so the LDS reads that produce it stay), store nothing
__device__ __forceinline__ void store_quad_nt(uint32_t *p, const u32x4h &v) {
    (void)p;
    asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
}
__device__ __forceinline__ void store_quad(uint32_t *p, const u32x4h &v) { store_quad_nt(p, v); }
__device__ __forceinline__ void store_word(uint32_t *p, uint32_t v) {
    (void)p;
    asm volatile("" ::"v"(v));
}
#else
__device__ __forceinline__ void store_quad_nt(uint32_t *p, const u32x4h &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4h *>(p));
}
__device__ __forceinline__ void store_quad(uint32_t *p, const u32x4h &v) { *reinterpret_cast<u32x4h *>(p) = v; }
__device__ __forceinline__ void store_word(uint32_t *p, uint32_t v) { *p = v; }
#endif
}  // namespace hooks

#ifdef RSORT_WG_TIMES
__device__ unsigned long long g_wg_times[8][2048][4];
__device__ unsigned long long g_wg_htimes[4][256][4];
#endif
}  // namespace rsort

#ifdef RSORT_WG_TIMES
#define RS_WG_T0 const unsigned long long wg_t0_ = __builtin_amdgcn_s_memrealtime();
#define RS_WG_TREC(TAB, SLOT, NB, B, E)                                                           \
    do {                                                                                          \
        __syncthreads();                                                                          \
        if (threadIdx.x == 0 && blockIdx.x < (NB)) {                                              \
            unsigned long long *p_ = TAB[SLOT][blockIdx.x];                                       \
            const unsigned long long hw_ = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   \
            const unsigned long long xc_ = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);  \
            p_[0] = wg_t0_;                                                                       \
            p_[1] = __builtin_amdgcn_s_memrealtime();                                             \
            p_[2] = (unsigned long long)(B) | (hw_ << 32);                                        \
            p_[3] = (unsigned long long)(E) | (xc_ << 32);                                        \
        }                                                                                         \
    } while (0)
#define RS_WG_T1 RS_WG_TREC(g_wg_times, (a.shift / BITS) & 7u, 2048u, cbeg, cend)
#define RS_WG_TH1 RS_WG_TREC(g_wg_htimes, (a.shift / 8u) & 3u, 256u, beg, end)
// (one translation unit includes this: rsort_kernels.hip, or a lab that includes it)
extern "C" __attribute__((visibility("default"), used)) int rsort_lab_wg_times(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rsort::g_wg_times), sizeof(rsort::g_wg_times)) == hipSuccess &&
                   hipMemcpyFromSymbol(host + 8 * 2048 * 4, HIP_SYMBOL(rsort::g_wg_htimes), sizeof(rsort::g_wg_htimes)) ==
                       hipSuccess
               ? 0
               : 6;
}
#else
#define RS_WG_T0
#define RS_WG_T1
#define RS_WG_TH1
#endif

#ifdef RSORT_STAMPS
#define RS_STAMP_DECL unsigned long long st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev_ = __builtin_amdgcn_s_memtime();
#define RS_STAMP(i)                                                   \
    do {                                                              \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        st_acc_[i] += now_ - st_prev_;                                \
        st_prev_ = now_;                                              \
    } while (0)
#define RS_STAMP_FLUSH()                                                                   \
    do {                                                                                   \
        if (threadIdx.x == 0 && a.stamps)                                                  \
            for (int i_ = 0; i_ < 8; ++i_) a.stamps[blockIdx.x * 8 + i_] = st_acc_[i_];    \
    } while (0)
#else
#define RS_STAMP_DECL
#define RS_STAMP(i)
#define RS_STAMP_FLUSH()
#endif
