// rsort_hooks.hpp -- the measurement hooks of the scatter and histogram kernels (rsort_kernels.hip).
//
// The library compiles every hook as the product behaviour below. A dev/ lab build (dev/build_variant.sh,
// dev/*_lab.hip) passes -DRSORT_LAB_HOOKS='"<path>/dev/lab_hooks.hpp"', which defines the same names with
// its instrumentation (per-workgroup start/end records, per-phase cycle stamps), its knob overrides
// (deferred-ranking batch sizes, counter replicas, occupancy) and its no-store floor build; nothing of
// dev/ is compiled into librsort.so. This is the only conditional the kernels' translation unit has.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef RSORT_LAB_HOOKS
#include RSORT_LAB_HOOKS
#else
namespace rsort {
namespace hooks {
// slots per issue batch of the deferred ranking (0: rank slot by slot), per kernel (DESIGN §3 "Deferred
// ranking": the clustered keys kernel 2, the plain keys kernel 0, the pairs kernel 4)
constexpr int kDeferKeysCl = 2;
constexpr int kDeferKeysPlain = 0;
constexpr int kDeferPairs = 4;
// replicas of every next-digit counter (k <= 4 line kernels; picked by lane % kNextReplicas)
constexpr int kNextReplicas = 8;
// minimum waves per SIMD asked of the register allocator by the 256-thread line kernels
constexpr int kLinesMinWavesSmall = 1;

typedef uint32_t u32x4h __attribute__((ext_vector_type(4)));
// the scatter kernels' global stores of their outputs (keys and values): whole 16-B quads, non-temporal or
// default policy, and single masked dwords
__device__ __forceinline__ void store_quad_nt(uint32_t *p, const u32x4h &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4h *>(p));
}
__device__ __forceinline__ void store_quad(uint32_t *p, const u32x4h &v) { *reinterpret_cast<u32x4h *>(p) = v; }
__device__ __forceinline__ void store_word(uint32_t *p, uint32_t v) { *p = v; }
}  // namespace hooks
}  // namespace rsort
// per-workgroup start / end records (rs_scatter_lines, the joint-count histograms) and per-phase cycle
// stamps (rs_scatter_pairs): none in the library
#define RS_WG_T0
#define RS_WG_T1
#define RS_WG_TH1
#define RS_STAMP_DECL
#define RS_STAMP(i)
#define RS_STAMP_FLUSH()
#endif
