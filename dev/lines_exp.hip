// Backs DESIGN §3 "Clustered input" and per-pass notes: rs_scatter_lines knob variants (OUTB2, COPY64, pad rows, rank candidates), uniform and Zipf passes 0..3.
// lines_exp.hip -- development harness (not part of the library): experimental copies of the
// keys-only rs_scatter_lines pass (cuda.radixsort_amd/csrc/rsort_kernels.hip) with knobs, timed
// against the library kernel on the same input and checked against its output.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cuda.radixsort_amd/csrc \
//         dev/lines_exp.hip -o dev/lines_exp && dev/lines_exp [log2n] [filter]
// -DLX_STAMPS: per-phase s_memtime stamps of wave 0 (diagnostic build).
//
// Knobs (template argument V, bit flags):
//   1  OUTB   output phase: every quad of a thread read from LDS first, then the segment records,
//             then the stores (the library reads quad -> waits -> record -> waits -> store)
//   2  RANK1  rank phase without the per-slot aggregation branch unless the previous tile of the
//             workgroup saw a per-wave digit count >= 32 (clustered input)
//   4  OUTB2  output phase in pairs of quads: both LDS reads, both records, both stores
//   8  SB16   staging in batches of 16 slots (all base reads, then all key writes)
//  16  PRIO   s_setprio 1 for waves 8..15 (the younger half, MI355X_MICROARCH.md item 4)
//  32  COPY64 carry copy with 8-B LDS accesses (ds_write_b128 costs 13 cycles, b64 6)
//  64  SB4    staging in batches of 4 slots
#define RSORT_LAB_HOOKS "../../dev/lab_hooks.hpp"
#include "../cuda.radixsort_amd/csrc/rsort_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include <vector>

using namespace rsort;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

#ifdef LX_STAMPS
#define LX_DECL unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = __builtin_amdgcn_s_memtime();
#define LX(i)                                                         \
    do {                                                              \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        st_acc[i] += now_ - st_prev;                                  \
        st_prev = now_;                                               \
    } while (0)
#define LX_FLUSH()                                                                \
    do {                                                                          \
        if (threadIdx.x == 0 && a.stamps)                                         \
            for (int i_ = 0; i_ < 8; ++i_) a.stamps[blockIdx.x * 8 + i_] = st_acc[i_]; \
    } while (0)
#else
#define LX_DECL
#define LX(i)
#define LX_FLUSH()
#endif

enum { kOutB = 1, kRank1 = 2, kOutB2 = 4, kSB16 = 8, kPrio = 16, kCopy64 = 32, kSB4 = 64, kHot2 = 128, kRuns = 256,
       kRunsAgg = 512, kGate = 1024, kGate128 = 2048, kGateW = 4096, kPad = 8192, kCopyI = 16384, kCopyR = 32768, kStSc1 = 65536, kStPlain = 131072, kStNtSc1 = 262144,
       kPeer = 524288, kPeerHot = 1048576 };

// kPeer: every lane finds the lanes sharing its digit (BITS ballots), the lowest of them adds the
// group's count with one returning add (no two lanes of an instruction on one counter), the
// others read the base from it (ds_bpermute) and add their rank in the group (mbcnt).
// kPeerHot: rank_add_hot's first-lane aggregation when >= 16 lanes share it, else kPeer.
template <int BITS>
__device__ __forceinline__ uint32_t rank_peer(uint32_t *cnt, uint32_t d) {
    uint32_t mlo, mhi;
    peer_mask<BITS>(d, mlo, mhi);
    const uint64_t m = ((uint64_t)mhi << 32) | mlo;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t o = 0;
    if (lane_id() == leader) o = atomicAdd(&cnt[d], (uint32_t)__popcll(m));
    const uint32_t base = (uint32_t)__shfl((int)o, (int)leader);
    return base + __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
}
template <int BITS>
__device__ __forceinline__ uint32_t rank_peer_hot(uint32_t *cnt, uint32_t d) {
    const uint32_t da = __builtin_amdgcn_readfirstlane(d);
    const uint64_t ma = __ballot(d == da);
    if (__popcll(ma) >= 16) return agg_add(cnt, d, da, ma);
    return rank_peer<BITS>(cnt, d);
}

// agg_add and rank_add_hot (kHot2) are the library's (rsort_kernels.hip)

// kRuns: runs of equal digits on consecutive lanes (every 16-lane row starts a run) -- only each
// run's first lane adds, the run's length; its lanes take base + offset (a DPP max scan per row)
template <bool AGG>
__device__ __forceinline__ uint32_t rank_runs(uint32_t *cnt, uint32_t d) {
    if constexpr (AGG) {
        const uint32_t da = __builtin_amdgcn_readfirstlane(d);
        const uint64_t ma = __ballot(d == da);
        if (__popcll(ma) >= 16) return agg_add(cnt, d, da, ma);
    }
    const uint32_t dp = (uint32_t)__builtin_amdgcn_update_dpp((int)~d, (int)d, 0x111, 0xf, 0xf, false);  // row_shr:1
    const bool head = dp != d;
    const uint64_t H = __ballot(head);
    if (__popcll(H) > 40) return atomicAdd(&cnt[d], 1u);
    const uint32_t lane = lane_id();
    const uint64_t above = H & ~((2ull << lane) - 1ull);
    const uint32_t next = above ? (uint32_t)__builtin_ctzll(above) : 64u;
    uint32_t o = 0;
    if (head) o = atomicAdd(&cnt[d], next - lane);
    uint32_t v = head ? ((lane << 16) | o) : 0u;
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    return (v & 0xFFFFu) + lane - (v >> 16);
}

template <int BITS, int THREADS, int KPT, int G, int V>
__global__ __launch_bounds__(THREADS) void lx_lines(ScatterArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int SEG = kWave * KPT;
    constexpr uint32_t T = THREADS * KPT;
    constexpr uint32_t TPD = THREADS / R;
    constexpr uint32_t CAP = T + (G - 1) * R;
    constexpr uint32_t QPL = G / 4;
    constexpr uint32_t MAXQ = (CAP / G) * QPL;                      // quads of a full staging area
    constexpr uint32_t QPT = (MAXQ + THREADS - 1) / THREADS;        // ... per thread
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    static_assert(R <= THREADS && TPD <= kWave && (G == 16 || G == 32), "geometry");

    __shared__ __attribute__((aligned(16))) uint32_t s_stage[CAP + R * G + 4];
    // kPad: per-wave counter rows R + 4 words apart, so the digit-group threads of step 2 (TPD = 4
    // threads per digit, rows 4 sub + i) hit 64 different banks (R apart they hit 16, 4-way)
    constexpr uint32_t RS = (V & kPad) ? R + 4 : R;
    __shared__ uint32_t s_cnt[W * RS + 1];
    __shared__ uint2 s_out[R];
    __shared__ uint2 s_flush[R];
    __shared__ uint32_t s_ws[W];
    __shared__ uint32_t s_clust[2];

    const uint32_t t = threadIdx.x;
    const uint32_t w = t / kWave;
    const uint32_t lane = lane_id();
    const uint32_t c = blockIdx.x;
    const Digit<BITS, kDigitShift> dig{a.shift, 0, nullptr};
    uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    uint32_t head = 0;
    if (a.bounds != nullptr && a.bounds[0] != 0u) {  // digit-group chunks (as the library kernel)
        const uint64_t b = a.bounds[1 + c];
        cend = a.bounds[2 + c];
        cbeg = b < cend ? (b & ~(uint64_t)(kWave - 1)) : cend;
        head = (uint32_t)(b < cend ? b - cbeg : 0);
    }

    const uint32_t d_own = t / TPD;
    const uint32_t sub = t % TPD;
    const bool leader = sub == 0;
    uint32_t g_run = 0, carry = 0, inv = 0;
    if (leader) {
        const uint32_t g = a.table[(uint64_t)d_own * a.num_chunks + c];
        carry = g & (G - 1u);
        inv = carry;
        g_run = g;
        const uint32_t ik = d_own << a.shift;
        for (uint32_t x = 0; x < inv; ++x) s_stage[CAP + d_own * G + x] = ik;
    }
    if (t < 2) s_clust[t] = 0;
    uint32_t clustered = 1;  // RANK1: the first tile checks
    uint32_t hotd = 0xFFFFFFFFu;  // HOT2: the wave's last aggregated digit
    uint32_t par = 0;

    const uint32_t base = w * SEG + lane;
    auto load_tile = [&](uint64_t tb, uint32_t (&k)[KPT]) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        uint32_t lb = base;
        asm volatile("" : "+v"(lb));
        const uint32_t *__restrict__ tk = a.kin + tb + lb;
        if (valid == T) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = __builtin_nontemporal_load(tk + j * kWave);
        } else {
            const uint32_t lim = valid > lb ? valid - lb : 0u;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool in = (uint32_t)(j * kWave) < lim;
                k[j] = in ? tk[j * kWave] : 0u;
            }
        }
    };

    auto store_quad = [&](uint32_t L, uint32_t q, const u32x4 &kv, const uint2 &info) {
        const uint32_t lo = (info.y >> 8) == L ? (info.y & 0xFFu) : 0u;
        const uint64_t gp = (uint64_t)(info.x + L * G + q);
        if (lo <= q) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(a.kout + gp);
            if constexpr ((V & kStSc1) != 0) {
                // write-through: the line leaves L2 at once, in issue order
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(kv) : "memory");
            } else if constexpr ((V & kStNtSc1) != 0) {
                asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(dst), "v"(kv) : "memory");
            } else if constexpr ((V & kStPlain) != 0) {
                *dst = kv;
            } else {
                __builtin_nontemporal_store(kv, dst);
            }
        } else {
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x)
                if (lo <= q + x) a.kout[gp + x] = kv[x];
        }
    };

    uint32_t key[KPT];
    if (cbeg < cend) load_tile(cbeg, key);
    __syncthreads();
    if constexpr ((V & kPrio) != 0) {
        if (w >= (uint32_t)W / 2) __builtin_amdgcn_s_setprio(1);
    }

    LX_DECL
    for (uint64_t tb = cbeg; tb < cend; tb += T) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        const bool full = valid == T && head == 0;
        const uint64_t nb = tb + T;
        uint32_t plim = valid > base ? valid - base : 0u;
        asm volatile("" : "+v"(plim));
        const bool h0 = base >= head;
        head = 0;
        LX(0);
#pragma unroll
        for (uint32_t i = lane; i < R; i += kWave) s_cnt[w * RS + i] = 0;
        uint32_t rk[(KPT + 1) / 2];
        uint32_t nkey[KPT];
        if (full) {
            if ((V & kRank1) && !clustered) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t dj = dig(key[j]);
                    const uint32_t r = atomicAdd(&s_cnt[w * RS + dj], 1u);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            } else if ((V & kGateW) && __builtin_expect([&] {
                           // this wave's tile is clustered: runs of equal digits on consecutive lanes
                           // in slots 0 and KPT / 2 (uniform keys: 1 lane in 256 matches its neighbour)
                           const uint32_t a0 = dig(key[0]), a1 = dig(key[KPT / 2]);
                           const uint32_t p0 = (uint32_t)__builtin_amdgcn_update_dpp((int)~a0, (int)a0, 0x111, 0xf, 0xf, false);
                           const uint32_t p1 = (uint32_t)__builtin_amdgcn_update_dpp((int)~a1, (int)a1, 0x111, 0xf, 0xf, false);
                           return __popcll(__ballot(p0 == a0)) + __popcll(__ballot(p1 == a1)) >= 16;
                       }(), 0)) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t dj = dig(key[j]);
                    const uint32_t r = rank_add_hot(&s_cnt[w * RS], dj, hotd);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            } else if ((V & kGate) && __builtin_expect(clustered != 0, 0)) {
                // clustered tiles (the previous tile had a per-wave digit count >= 32 / 128): a
                // second aggregation candidate, the wave's last aggregated digit
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t dj = dig(key[j]);
                    const uint32_t r = rank_add_hot(&s_cnt[w * RS], dj, hotd);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            } else {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t dj = dig(key[j]);
                    uint32_t r;
                    if constexpr ((V & kPeer) != 0) r = rank_peer<BITS>(&s_cnt[w * RS], dj);
                    else if constexpr ((V & kPeerHot) != 0) r = rank_peer_hot<BITS>(&s_cnt[w * RS], dj);
                    else if constexpr ((V & kHot2) != 0) r = rank_add_hot(&s_cnt[w * RS], dj, hotd);
                    else if constexpr ((V & kRuns) != 0) r = rank_runs<false>(&s_cnt[w * RS], dj);
                    else if constexpr ((V & kRunsAgg) != 0) r = rank_runs<true>(&s_cnt[w * RS], dj);
                    else r = rank_add(&s_cnt[w * RS], dj);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = dig(key[j]);
                uint32_t r = 0;
                if ((uint32_t)(j * kWave) < plim && (j != 0 || h0)) r = atomicAdd(&s_cnt[w * RS + d], 1u);
                rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
            }
        }
        if (nb < cend) load_tile(nb, nkey);
        __syncthreads();
        LX(1);

        constexpr uint32_t WPT = (W >= (int)TPD) ? W / TPD : 1;
        uint32_t part = 0;
        uint32_t wx[WPT];
        bool hot = false;
        if (sub < (uint32_t)W) {
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i) {
                const uint32_t v = sub * WPT + i;
                wx[i] = v < (uint32_t)W ? s_cnt[v * RS + d_own] : 0u;
                part += wx[i];
                hot |= wx[i] >= ((V & kGate128) ? 128u : 32u);
            }
        }
        if constexpr ((V & (kRank1 | kGate)) != 0) {
            // slot par: set by any wave that saw a hot per-wave digit count, read after the barrier
            // below; slot par ^ 1 is reset for the next tile (its readers are a barrier behind)
            if (__ballot(hot) != 0 && lane == 0) s_clust[par] = 1;
            if (t == 0) s_clust[par ^ 1u] = 0;
        }
        uint32_t gpre, cnt;
        group_scan<TPD>(part, sub, gpre, cnt);
        uint32_t wcnt = 0, A = 0, e = 0;
        if (leader) {
            A = g_run - carry;
            e = g_run + cnt;
            wcnt = max(A, e & ~(uint32_t)(G - 1)) - A;
        }
        uint32_t nseg;
        const uint32_t S = block_excl_scan1<THREADS>(wcnt, s_ws, nseg);
        LX(2);
        const uint32_t gS = group_lane<TPD>(S, 0), gw = group_lane<TPD>(wcnt, 0);
        const uint32_t gA = group_lane<TPD>(A, 0), gc = group_lane<TPD>(carry, 0), ginv = group_lane<TPD>(inv, 0);
        {
            const uint32_t d = d_own;
            if (sub < (uint32_t)W) {
                uint32_t acc = gS + gc + gpre;
#pragma unroll
                for (uint32_t i = 0; i < WPT; ++i) {
                    const uint32_t v = sub * WPT + i;
                    if (v < (uint32_t)W) s_cnt[v * RS + d] = acc | ((gS + gw) << 16);
                    acc += wx[i];
                }
            }
            constexpr uint32_t CB = G / TPD;
            static_assert(G % TPD == 0 && CB % 4 == 0, "quad carries");
            const uint32_t x0 = sub * CB;
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            if ((V & kCopyR) != 0) {
                // 8-B units, each thread's 4 units rotated by the digit: the 16 digits of a wave
                // then touch different banks (segment heads and carry areas sit at 0 or 32 mod 64)
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                constexpr uint32_t UPT = G / 2 / TPD;  // units per thread
                if (gw > 0) {
                    const uint32_t rot = d & (G / 2 - 1);
                    u32x2 ck[UPT];
#pragma unroll
                    for (uint32_t i = 0; i < UPT; ++i) {
                        const uint32_t u = (sub + TPD * i + rot) & (G / 2 - 1);
                        ck[i] = *reinterpret_cast<const u32x2 *>(&s_stage[CAP + d * G + 2 * u]);
                    }
#pragma unroll
                    for (uint32_t i = 0; i < UPT; ++i) {
                        const uint32_t x = 2 * ((sub + TPD * i + rot) & (G / 2 - 1));
                        if (x + 2 <= gc) *reinterpret_cast<u32x2 *>(&s_stage[gS + x]) = ck[i];
                        else if (x < gc) s_stage[gS + x] = ck[i][0];
                    }
                }
            } else if ((V & kCopyI) != 0) {
                // interleaved dword copy: the group's lanes take consecutive slots (no bank conflicts)
                if (gw > 0) {
                    uint32_t ck[G / TPD];
#pragma unroll
                    for (uint32_t i = 0; i < G / TPD; ++i) {
                        const uint32_t x = sub + i * TPD;
                        ck[i] = s_stage[CAP + d * G + x];
                    }
#pragma unroll
                    for (uint32_t i = 0; i < G / TPD; ++i) {
                        const uint32_t x = sub + i * TPD;
                        if (x < gc) s_stage[gS + x] = ck[i];
                    }
                }
            } else if ((V & kCopy64) != 0 && gw > 0 && x0 < gc) {
                u32x2 ck[CB / 2];
#pragma unroll
                for (uint32_t i = 0; i < CB / 2; ++i)
                    ck[i] = *reinterpret_cast<const u32x2 *>(&s_stage[CAP + d * G + x0 + 2 * i]);
#pragma unroll
                for (uint32_t i = 0; i < CB / 2; ++i) {
                    const uint32_t x = x0 + 2 * i;
                    if (x + 2 <= gc) *reinterpret_cast<u32x2 *>(&s_stage[gS + x]) = ck[i];
                    else if (x < gc) s_stage[gS + x] = ck[i][0];
                }
            } else if (gw > 0 && x0 < gc) {
                u32x4 ck[CB / 4];
#pragma unroll
                for (uint32_t i = 0; i < CB / 4; ++i)
                    ck[i] = *reinterpret_cast<const u32x4 *>(&s_stage[CAP + d * G + x0 + 4 * i]);
#pragma unroll
                for (uint32_t i = 0; i < CB / 4; ++i) {
                    const uint32_t x = x0 + 4 * i;
                    if (x + 4 <= gc) {
                        *reinterpret_cast<u32x4 *>(&s_stage[gS + x]) = ck[i];
                    } else if (x < gc) {
#pragma unroll
                        for (uint32_t e2 = 0; e2 < 4; ++e2)
                            if (x + e2 < gc) s_stage[gS + x + e2] = ck[i][e2];
                    }
                }
            }
            if (leader) {
                s_out[d] = make_uint2(gA - gS, ((gS / G) << 8) | ginv);
                if (gw > 0) inv = 0;
                carry = e - (A + gw);
                g_run = e;
                if (nb >= cend) s_flush[d] = make_uint2(g_run - carry, inv | (carry << 8));
            }
        }
        LX(3);
        __syncthreads();
        if constexpr ((V & (kRank1 | kGate)) != 0) {
            clustered = s_clust[par];
            par ^= 1u;
        }
        LX(4);

        constexpr int SB = (V & kSB16) ? KPT : (V & kSB4) ? 4 : (KPT < 8 ? KPT : 8);
#pragma unroll
        for (int j0 = 0; j0 < KPT; j0 += SB) {
            uint32_t pp[SB], ll[SB], dd[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                asm volatile("" : "+v"(key[j]));
                dd[u] = dig(key[j]);
                const uint32_t bl = s_cnt[w * RS + dd[u]];
                pp[u] = (bl & 0xFFFFu) + ((j & 1) ? (rk[j / 2] >> 16) : (rk[j / 2] & 0xFFFFu));
                ll[u] = bl >> 16;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                uint32_t idx = pp[u] < ll[u] ? pp[u] : CAP + dd[u] * G + (pp[u] - ll[u]);
                if (!(full || ((uint32_t)(j * kWave) < plim && (j != 0 || h0)))) idx = CAP + R * G;
                s_stage[idx] = key[j];
            }
        }
        __syncthreads();
        LX(5);

        const uint32_t nq = (nseg / G) * QPL;
        if constexpr ((V & kOutB) != 0) {
            u32x4 kv[QPT];
            uint2 info[QPT];
#pragma unroll
            for (uint32_t i = 0; i < QPT; ++i) {
                const uint32_t item = t + i * THREADS;
                if (item < nq) kv[i] = *reinterpret_cast<const u32x4 *>(&s_stage[(item / QPL) * G + (item % QPL) * 4]);
            }
#pragma unroll
            for (uint32_t i = 0; i < QPT; ++i) {
                const uint32_t item = t + i * THREADS;
                if (item < nq) info[i] = s_out[dig(kv[i].x)];
            }
#pragma unroll
            for (uint32_t i = 0; i < QPT; ++i) {
                const uint32_t item = t + i * THREADS;
                if (item < nq) store_quad(item / QPL, (item % QPL) * 4, kv[i], info[i]);
            }
        } else if constexpr ((V & kOutB2) != 0) {
            for (uint32_t item = t; item < nq; item += 2 * THREADS) {
                const uint32_t i2 = item + THREADS;
                const bool two = i2 < nq;
                const u32x4 kv0 = *reinterpret_cast<const u32x4 *>(&s_stage[(item / QPL) * G + (item % QPL) * 4]);
                u32x4 kv1 = kv0;
                if (two) kv1 = *reinterpret_cast<const u32x4 *>(&s_stage[(i2 / QPL) * G + (i2 % QPL) * 4]);
                const uint2 in0 = s_out[dig(kv0.x)];
                const uint2 in1 = s_out[dig(kv1.x)];
                store_quad(item / QPL, (item % QPL) * 4, kv0, in0);
                if (two) store_quad(i2 / QPL, (i2 % QPL) * 4, kv1, in1);
            }
        } else {
#pragma unroll 2
            for (uint32_t item = t; item < nq; item += THREADS) {
                const uint32_t L = item / QPL, q = (item % QPL) * 4u;
                const u32x4 kv = *reinterpret_cast<const u32x4 *>(&s_stage[L * G + q]);
                store_quad(L, q, kv, s_out[dig(kv.x)]);
            }
        }
        LX(6);
#pragma unroll
        for (int j = 0; j < KPT; ++j) key[j] = nkey[j];
    }
    if (cbeg < cend) {
        for (uint32_t item = t; item < R * G; item += THREADS) {
            const uint2 fl = s_flush[item / G];
            const uint32_t x = item % G;
            if ((fl.y & 0xFFu) <= x && x < (fl.y >> 8)) a.kout[(uint64_t)fl.x + x] = s_stage[CAP + item];
        }
    }
    LX_FLUSH();
}

// reads every stride-th word of buf (keeps a sum so the loads stay)
__global__ void touch(const uint32_t *buf, uint64_t n, uint64_t stride, unsigned long long *sink) {
    uint32_t acc = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * stride; i < n; i += (uint64_t)gridDim.x * blockDim.x * stride)
        acc += buf[i];
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

__global__ void count_mismatch(const uint32_t *a, const uint32_t *b, uint64_t n, unsigned long long *bad) {
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        local += a[i] != b[i];
    if (local) atomicAdd(bad, local);
}

struct Ctx {
    uint64_t n;
    uint32_t *keys, *out, *ref, *table, *bsums, *joint, *bounds;
    bool groups = false;  // LX_GROUPS=1 (with LX_PASS=1): pass 1 on the digit-0 groups
    unsigned long long *bad, *stamps;
    int cus;
    hipEvent_t e0, e1;
    bool have_ref = false;
};

static const char *g_filter = nullptr;
static int g_shift = 0;
static int g_disturb = 0;

template <int BITS, int THREADS, int KPT, typename K>
void run(Ctx &c, const char *name, K kern, int shift, int reps = 10) {
    if (g_filter && !strstr(name, g_filter)) return;
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kern, THREADS, 0));
    const uint64_t T = (uint64_t)THREADS * KPT;
    const uint64_t tiles = (c.n + T - 1) / T;
    const uint64_t target = (uint64_t)c.cus * bpc;
    const uint64_t tpc = (tiles + target - 1) / target;
    const uint64_t chunks = (tiles + tpc - 1) / tpc;
    HistArgs h{};
    h.keys = c.keys;
    h.table = c.table;
    h.n = c.n;
    h.chunk_keys = tpc * T;
    h.num_chunks = (uint32_t)chunks;
    h.shift = shift;
    h.vec = 1;
    h.split = 1;
    if (c.groups) {  // the table is the joint counts (copy mode), the chunks the groups
        h.bounds = c.bounds;
        h.copy_src = c.joint;
    }
    CK(launch_histogram(BITS, kDigitShift, h, 0));
    ScanArgs s{};
    s.table = c.table;
    s.block_sums = c.bsums;
    s.m = (uint64_t)chunks << BITS;
    s.nblocks = (uint32_t)((s.m + kScanSegment - 1) / kScanSegment);
    CK(launch_scan(s, 0));
    ScatterArgs a{};
    a.kin = c.keys;
    a.kout = c.out;
    a.table = c.table;
    a.n = c.n;
    a.chunk_keys = tpc * T;
    a.num_chunks = (uint32_t)chunks;
    a.shift = shift;
    a.stamps = c.stamps;
    if (c.groups) a.bounds = c.bounds;
    CK(hipMemset(c.out, 0, c.n * 4));
    kern<<<chunks, THREADS>>>(a);
    CK(hipDeviceSynchronize());
    float ms = 0;
    if (g_disturb == 0) {
        CK(hipEventRecord(c.e0, 0));
        for (int i = 0; i < reps; ++i) kern<<<chunks, THREADS>>>(a);
        CK(hipEventRecord(c.e1, 0));
        CK(hipEventSynchronize(c.e1));
        CK(hipGetLastError());
        CK(hipEventElapsedTime(&ms, c.e0, c.e1));
        ms /= reps;
    } else {
        // LX_DISTURB: before each timed launch, read another 4 GiB buffer (caches and TLBs hold
        // other data), then 2: touch one word per 64 KiB of the input, 3: read the whole input
        for (int i = 0; i < reps; ++i) {
            touch<<<4096, 256>>>(c.ref, c.n, 1, c.bad + 1);
            if (g_disturb == 2) touch<<<4096, 256>>>(c.keys, c.n, 16384, c.bad + 1);
            if (g_disturb == 3) touch<<<4096, 256>>>(c.keys, c.n, 1, c.bad + 1);
            CK(hipEventRecord(c.e0, 0));
            kern<<<chunks, THREADS>>>(a);
            CK(hipEventRecord(c.e1, 0));
            CK(hipEventSynchronize(c.e1));
            float one = 0;
            CK(hipEventElapsedTime(&one, c.e0, c.e1));
            ms += one / reps;
        }
    }
    unsigned long long bad = 0;
    if (!c.have_ref) {
        CK(hipMemcpy(c.ref, c.out, c.n * 4, hipMemcpyDeviceToDevice));
        c.have_ref = true;
    } else {
        CK(hipMemset(c.bad, 0, 8));
        count_mismatch<<<4096, 256>>>(c.out, c.ref, c.n, c.bad);
        CK(hipMemcpy(&bad, c.bad, 8, hipMemcpyDeviceToHost));
    }
    printf("%-40s chunks=%-5llu tpc=%-4llu %8.3f ms %7.1f GB/s %5.1f%%  mismatch=%llu\n", name,
           (unsigned long long)chunks, (unsigned long long)tpc, ms, 8.0 * c.n / ms / 1e6, 8.0 * c.n / ms / 1e6 / 80.0, bad);
#ifdef LX_STAMPS
    std::vector<unsigned long long> st(chunks * 8);
    CK(hipMemcpy(st.data(), c.stamps, chunks * 8 * 8, hipMemcpyDeviceToHost));
    double sum[8] = {0};
    for (uint64_t b = 0; b < chunks; ++b)
        for (int i = 0; i < 8; ++i) sum[i] += st[b * 8 + i];
    const char *names[8] = {"loop", "1:rank+bar", "2:scan", "2:bases+carry", "2:bar", "3:stage+bar", "4:out", "-"};
    printf("    cycles per tile (wave 0):");
    for (int i = 0; i < 7; ++i) printf(" %s=%.0f", names[i], sum[i] / chunks / tpc);
    printf("\n");
    // the slowest chunk sets the kernel time (one workgroup per CU, all resident at once)
    uint64_t worst = 0;
    double wt = 0;
    for (uint64_t b = 0; b < chunks; ++b) {
        double tot = 0;
        for (int i = 0; i < 7; ++i) tot += st[b * 8 + i];
        if (tot > wt) { wt = tot; worst = b; }
    }
    printf("    slowest chunk %llu (%.2fx the mean):", (unsigned long long)worst,
           wt / ((sum[0] + sum[1] + sum[2] + sum[3] + sum[4] + sum[5] + sum[6]) / chunks));
    for (int i = 0; i < 7; ++i) printf(" %s=%.0f", names[i], (double)st[worst * 8 + i] / tpc);
    printf("\n");
#endif
    fflush(stdout);
}

int main(int argc, char **argv) {
    Ctx c{};
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    g_filter = argc > 2 ? argv[2] : nullptr;
    c.n = 1ull << lg;
    CK(hipDeviceGetAttribute(&c.cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&c.keys, c.n * 4));
    CK(hipMalloc(&c.out, c.n * 4));
    CK(hipMalloc(&c.ref, c.n * 4));
    CK(hipMalloc(&c.table, (c.n / 1024 + 65536) * 4 * 16));
    CK(hipMalloc(&c.bsums, 1 << 24));
    CK(hipMalloc(&c.bad, 16));
    CK(hipMalloc(&c.stamps, 65536 * 8 * 8));
    CK(hipEventCreate(&c.e0));
    CK(hipEventCreate(&c.e1));
    const bool zipf = getenv("LX_ZIPF") != nullptr;
    if (zipf) {
        // Zipf(1.0) over 2^20 ranks, key = fmix32(rank) (bench.py --dist zipf, tests/_util.py)
        const int ranks = 1 << 20;
        std::vector<double> cum(ranks);
        double acc = 0;
        for (int r = 0; r < ranks; ++r) cum[r] = (acc += 1.0 / (r + 1.0));
        std::vector<uint32_t> cdf(ranks);
        for (int r = 0; r < ranks; ++r) {
            const double t = floor(cum[r] / acc * 4294967296.0);
            cdf[r] = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
        }
        cdf[ranks - 1] = 0xFFFFFFFFu;
        uint32_t *d_cdf = nullptr;
        CK(hipMalloc(&d_cdf, ranks * 4));
        CK(hipMemcpy(d_cdf, cdf.data(), ranks * 4, hipMemcpyHostToDevice));
        CK(launch_gen_zipf(c.keys, c.n, 0x5EED, d_cdf, ranks, 0));
    } else {
        CK(launch_gen_uniform(c.keys, c.n, 0x5EED, 0));
    }
    CK(hipDeviceSynchronize());
    // LX_PASS=p: the input of pass p of a sort (p library passes over fixed chunks first)
    const int npre = getenv("LX_PASS") ? atoi(getenv("LX_PASS")) : 0;
    g_disturb = getenv("LX_DISTURB") ? atoi(getenv("LX_DISTURB")) : 0;
    CK(hipMalloc(&c.joint, 65536 * 4));
    CK(hipMalloc(&c.bounds, 1024 * 4));
    if (getenv("LX_GROUPS") && npre == 1) {
        // joint counts (digit 0, digit 1) of the input and the digit-0 group bounds (library kernels)
        CK(hipMemset(c.joint, 0, 65536 * 4));
        HistArgs hj{};
        hj.keys = c.keys; hj.table = c.table; hj.n = c.n; hj.chunk_keys = c.n / 256; hj.num_chunks = 256;
        hj.shift = 0; hj.vec = 1; hj.split = 1; hj.joint = c.joint;
        CK(launch_histogram_joint(hj, 0));
        CK(launch_joint_bounds(c.joint, nullptr, c.bounds, nullptr, nullptr, c.n, c.n / 256 + 16384, 0, 0, 0));
        c.groups = true;
    }
    for (int i = 0; i < npre; ++i) {
        HistArgs h{};
        h.keys = c.keys; h.table = c.table; h.n = c.n; h.chunk_keys = c.n / 256; h.num_chunks = 256;
        h.shift = 8 * i; h.vec = 1; h.split = 1;
        CK(launch_histogram(8, kDigitShift, h, 0));
        ScanArgs sa{};
        sa.table = c.table; sa.block_sums = c.bsums; sa.m = 256 * 256; sa.nblocks = (uint32_t)((sa.m + kScanSegment - 1) / kScanSegment);
        CK(launch_scan(sa, 0));
        ScatterArgs a{};
        a.kin = c.keys; a.kout = c.out; a.table = c.table; a.n = c.n; a.chunk_keys = c.n / 256; a.num_chunks = 256;
        a.shift = 8 * i;
        rs_scatter_lines<8, 1024, 16, 32, false, kDigitShift, 3><<<256, 1024>>>(a);
        CK(hipMemcpy(c.keys, c.out, c.n * 4, hipMemcpyDeviceToDevice));
    }
    g_shift = 8 * npre;
    CK(hipDeviceSynchronize());
    printf("n=%llu cus=%d keys=%s pass=%d%s\n", (unsigned long long)c.n, c.cus, zipf ? "zipf" : "uniform", npre,
           c.groups ? " groups" : "");
    constexpr int OC = kOutB2 | kCopy64;
    for (int rep = 0; rep < 2; ++rep) {
        run<8, 1024, 16>(c, "lib rs_scatter_lines<8,1024,16,32,nt>", rs_scatter_lines<8, 1024, 16, 32, false, kDigitShift, 3>, g_shift);
        run<8, 1024, 16>(c, "lx base", lx_lines<8, 1024, 16, 32, 0>, g_shift);
        run<8, 1024, 16>(c, "lx outb2+copy64", lx_lines<8, 1024, 16, 32, OC>, g_shift);
        run<8, 1024, 16>(c, "lx pad", lx_lines<8, 1024, 16, 32, OC | kPad>, g_shift);
        run<8, 1024, 16>(c, "lx pad sc1", lx_lines<8, 1024, 16, 32, OC | kPad | kStSc1>, g_shift);
        run<8, 1024, 16>(c, "lx pad nt sc1", lx_lines<8, 1024, 16, 32, OC | kPad | kStNtSc1>, g_shift);
        run<8, 1024, 16>(c, "lx pad plain", lx_lines<8, 1024, 16, 32, OC | kPad | kStPlain>, g_shift);
        run<8, 1024, 16>(c, "lib CL rs_scatter_lines<...,3,1>", rs_scatter_lines<8, 1024, 16, 32, false, kDigitShift, 3, 1>, g_shift);
        run<8, 1024, 16>(c, "lx pad hot2", lx_lines<8, 1024, 16, 32, OC | kPad | kHot2>, g_shift);
        run<8, 1024, 16>(c, "lx pad runs", lx_lines<8, 1024, 16, 32, OC | kPad | kRuns>, g_shift);
        run<8, 1024, 16>(c, "lx pad runsagg", lx_lines<8, 1024, 16, 32, OC | kPad | kRunsAgg>, g_shift);
        run<8, 1024, 16>(c, "lx pad peer", lx_lines<8, 1024, 16, 32, OC | kPad | kPeer>, g_shift);
        run<8, 1024, 16>(c, "lx pad peerhot", lx_lines<8, 1024, 16, 32, OC | kPad | kPeerHot>, g_shift);
    }
    return 0;
}
