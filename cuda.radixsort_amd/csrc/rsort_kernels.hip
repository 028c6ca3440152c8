// rsort_kernels.hip -- the per-digit pass of the LSD radix sort, hand-written for gfx950.
//
// One pass (reference Parallel7.cu:561-623) is three launches:
//
//   rs_histogram  per-chunk k-bit histogram in LDS, written COLUMN-major [digit][chunk]
//                 (reference: histogramKernel P7:318-343 + the transpose of P7:596 folded into
//                 the store, so no transpose kernel is needed)
//   rs_scan_*     exclusive scan of that column-major table, fully on device
//                 (reference: scanBlocks/addScannedBlockSums P7:408-528 + transpose back
//                 P7:598; the per-pass D2H/H2D block-sum round trip P7:514-519 is gone)
//   rs_scatter    per tile: block-local stable sort by the digit in LDS + global rank +
//                 scatter (reference: sortLocallyDataBlocks P7:193-251 and scatterKernel
//                 P7:253-304, fused: the tile is read once and written once)
//
// A workgroup owns a CHUNK of `tiles_per_chunk` consecutive tiles of kTileKeys keys and
// walks them in order, carrying the running global offset of every digit in registers:
// the table is chunk x digit (not tile x digit as in P7), so it stays tiny and L2-resident
// and each digit's output run continues where the previous tile of the same workgroup
// stopped (partial cache lines complete inside one CU's L2 before write-back).
//
// Local rank (the "block-local 1-bit split sort" of the north star), three interchangeable
// algorithms giving the same unique stable order (public rsort_rank_algo -> internal RankAlgo):
//   RSORT_RANK_MATCH (default) -> kRankAtomic: count first (per-wave LDS digit counters), scan
//               them into tile positions, then ONE returning ds_add per key: gfx950 serves the
//               lanes of one ds_add_rtn_u32 that hit the same address in ascending lane order,
//               so the returned value IS the key's stable position (rank_add / rank_add_hot;
//               rs_lane_order_probe re-checks the premise once per device and the library falls
//               back to kRankCount when it fails).
//   RSORT_RANK_BALLOT -> kRankCount: the same count-first scheme with a wave64 ballot peer match
//               (k ballots build the mask of lanes holding the same digit; rank-in-wave =
//               popcount(mask & lanes-below) + the per-wave counter bumped by one lane).
//   RSORT_RANK_SPLIT -> kRankSplit: k successive stable 1-bit splits (the reference's
//               P5:79-159 / P7:79-191 algorithm), each a ballot/popcount block scan + one LDS
//               permutation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "rsort_hooks.hpp"
#include "rsort_internal.hpp"

namespace rsort {

// ------------------------------------------------------------------------------ kernel names
// Which scatter kernels a sort actually launched (rsort_scatter_kernels_used, bench.py's line):
// every kernel pointer the dispatch below hands out goes through reg_lines<...>() / reg_scatter<...>(),
// which
// records the instantiation's name (its template arguments) once; launch_scatter notes the pointers
// it launches.
namespace {
std::mutex g_kn_mu;
std::vector<std::pair<const void *, std::string>> g_kn_names;  // every registered kernel
std::vector<const void *> g_kn_lines;                           // ... of them the whole-line kernels
std::vector<const void *> g_kn_used;                           // launched since the last reset

void register_kernel(const void *fn, const char *name, bool lines = false) {
    std::lock_guard<std::mutex> g(g_kn_mu);
    g_kn_names.emplace_back(fn, std::string(name));
    if (lines) g_kn_lines.push_back(fn);
}

bool is_line_kernel(const void *fn) {
    std::lock_guard<std::mutex> g(g_kn_mu);
    for (const void *x : g_kn_lines)
        if (x == fn) return true;
    return false;
}

void note_used(const void *fn) {
    std::lock_guard<std::mutex> g(g_kn_mu);
    for (const void *u : g_kn_used)
        if (u == fn) return;
    g_kn_used.push_back(fn);
}
}  // namespace

size_t scatter_kernels_used(char *buf, size_t len, int reset) {
    std::lock_guard<std::mutex> g(g_kn_mu);
    std::string out;
    for (const void *u : g_kn_used) {
        std::string nm = "?";
        for (auto &kv : g_kn_names)
            if (kv.first == u) nm = kv.second;
        if (!out.empty()) out += ";";
        out += nm;
    }
    if (reset) g_kn_used.clear();
    if (buf && len > 0) {
        const size_t m = std::min(len - 1, out.size());
        memcpy(buf, out.data(), m);
        buf[m] = '\0';
    }
    return out.size();
}


// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

// Lane count of a wave-uniform mask as an opaque 32-bit scalar. `__popcll(m) < c` is folded into a
// 64-bit unsigned compare of the i64 popcount, which the SALU cannot do (no s_cmp_lt_u64): it went
// to the VALU (v_cmp_lt_u64 on SGPR operands) on every key of the rank loops. s_bcnt1 into a 32-bit
// SGPR keeps the test on the SALU (s_cmp + s_cbranch_scc). s_bcnt1 also writes SCC: declared, or the
// compiler may place it between another compare and the branch on that compare (it did, round 6: a
// tile's rank-check test `tno & 7` branched on this count instead).
__device__ __forceinline__ uint32_t wave_count(uint64_t m) {
    uint32_t c;
    asm("s_bcnt1_i32_b64 %0, %1" : "=s"(c) : "s"(m) : "scc");
    return c;
}

// Lane-ordered returning LDS add of 1 to cnt[d] for every lane of a wave (the kRankAtomic
// premise: same-address lanes are served in lane order, so lane l gets old + #lower lanes with
// digit d). Same-address lanes serialise in the LDS (about 2 cycles each: 127 cycles when all 64
// lanes share a counter, dev/lds_rate_lab.hip) and clustered input -- runs of equal keys, as
// every pass after the first sees for duplicate-heavy data -- does exactly that. So when the
// digit held by the first active lane is common (>= 16 lanes: a run crossing the slot's start,
// or a slot inside one run), it is added once, by that lane, for all its lanes, whose ranks come
// from mbcnt; a run that starts inside the slot is served lane by lane (once per run). Uniform
// data pays one compare, a popcount and a scalar branch. Exact under any exec mask.
__device__ __forceinline__ uint32_t rank_add(uint32_t *cnt, uint32_t d) {
    const uint32_t da = __builtin_amdgcn_readfirstlane(d);
    const uint64_t ma = __ballot(d == da);
    if (wave_count(ma) < 16) return atomicAdd(&cnt[d], 1u);
    const uint32_t la = (uint32_t)__builtin_ctzll(ma);
    uint32_t o = 0;
    if (d != da) o = atomicAdd(&cnt[d], 1u);
    if (lane_id() == la) o = atomicAdd(&cnt[da], (uint32_t)__popcll(ma));
    const uint32_t base = __builtin_amdgcn_readlane(o, la);
    return d == da ? base + (uint32_t)__popcll(ma & lanes_below()) : o;
}

// Non-returning form for histograms (same aggregation; exact under any exec mask).
__device__ __forceinline__ void count_add(uint32_t *cnt, uint32_t d, uint32_t inc = 1u) {
    const uint32_t da = __builtin_amdgcn_readfirstlane(d);
    const uint64_t ma = __ballot(d == da);
    if (wave_count(ma) < 16) {
        atomicAdd(&cnt[d], inc);
        return;
    }
    if (d != da) atomicAdd(&cnt[d], inc);
    if (lane_id() == (uint32_t)__builtin_ctzll(ma)) atomicAdd(&cnt[da], inc * (uint32_t)__popcll(ma));
}

// One returning add for all lanes of a wave: the lanes whose digit is c (mask m) are served by the
// first of them, adding their count, and get base + their rank among m (mbcnt); every other lane
// adds 1 (lane-ordered). One ds_add_rtn instruction.
__device__ __forceinline__ uint32_t agg_add(uint32_t *cnt, uint32_t d, uint32_t c, uint64_t m) {
    const uint32_t la = (uint32_t)__builtin_ctzll(m);
    const bool mine = d == c;
    uint32_t o = 0;
    if (!mine || lane_id() == la) o = atomicAdd(&cnt[d], mine ? (uint32_t)__popcll(m) : 1u);
    const uint32_t base = __builtin_amdgcn_readlane(o, la);
    return mine ? base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) : o;
}

// rank_add for clustered input (the clustered-pass kernels, rs_scatter_lines<..., CL = 1>): when the
// first lane's digit is not common, the wave's last aggregated digit (`hot`, wave-uniform) is the
// second candidate -- a run of a hot key covers many consecutive slots, but where it holds ~2/3 of
// a slot's lanes the first lane holds another key a third of the time, and then ~40 lanes would
// serialise on one counter (dev/lines_exp.hip, Zipf pass 1: 2.35 -> 2.16 ms; it costs ~12 % on
// unclustered input, so only the clustered kernels use it).
__device__ __forceinline__ uint32_t rank_add_hot(uint32_t *cnt, uint32_t d, uint32_t &hot) {
    const uint32_t da = __builtin_amdgcn_readfirstlane(d);
    const uint64_t ma = __ballot(d == da);
    if (wave_count(ma) >= 16) {
        hot = da;
        return agg_add(cnt, d, da, ma);
    }
    const uint64_t mh = __ballot(d == hot);
    if (wave_count(mh) >= 8) return agg_add(cnt, d, hot, mh);
    return atomicAdd(&cnt[d], 1u);
}

// rank_add_hot in two halves, so a tile's KPT slots issue their returning adds back to back and
// wait for the LDS once: hot_issue picks the slot's aggregated digit c (~0u: none) and its lanes m
// exactly as rank_add_hot and issues the slot's one add; hot_rank, after every slot is issued, turns
// the returns into ranks (the aggregated lanes read their leader's return).
template <bool HOT>
__device__ __forceinline__ uint32_t hot_issue(uint32_t *cnt, uint32_t d, uint32_t &hot, uint32_t &c, uint64_t &m) {
    const uint32_t da = __builtin_amdgcn_readfirstlane(d);
    const uint64_t ma = __ballot(d == da);
    if (wave_count(ma) >= 16) {
        hot = da;
        c = da;
        m = ma;
    } else if (!HOT) {
        c = 0xFFFFFFFFu;
        m = 0ull;
    } else {
        const uint64_t mh = __ballot(d == hot);
        const bool agg = wave_count(mh) >= 8;
        c = agg ? hot : 0xFFFFFFFFu;
        m = agg ? mh : 0ull;
    }
    const bool mine = d == c;
    uint32_t o = 0;
    if (!mine || lane_id() == (uint32_t)__builtin_ctzll(m)) o = atomicAdd(&cnt[d], mine ? (uint32_t)__popcll(m) : 1u);
    return o;
}
__device__ __forceinline__ uint32_t hot_rank(uint32_t o, uint32_t d, uint32_t c, uint64_t m) {
    if (c == 0xFFFFFFFFu) return o;
    const uint32_t base = __builtin_amdgcn_readlane(o, (uint32_t)__builtin_ctzll(m));
    return d == c ? base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) : o;
}

// Row stride of per-wave digit counters [wave][digit] read column-wise by digit groups: TPD threads
// per digit, thread `sub` taking rows sub * WPT .. + WPT - 1. With rows R apart (R a multiple of
// 64) the TPD threads of a digit hit one bank; a stride with WPT * RS = 64 / TPD (mod 64) puts the
// 64 / TPD digits x TPD threads of a wave on 64 different banks (k = 8, 1024 threads: 260;
// dev/lines_exp.hip "lx pad": step 2 2.1K -> 1.75K cycles per tile, C3 pass -1.5 %). Groups wider
// than the wave count (WPT = 0 here) read one row per thread and keep R.
template <uint32_t R, uint32_t TPD, uint32_t WPT>
constexpr uint32_t counter_stride() {
    if (TPD < 2 || WPT == 0 || 64 % TPD != 0) return R;
    for (uint32_t p = 0; p < 64; ++p)
        if (((R + p) * WPT) % 64 == (64 / TPD) % 64) return R + p;
    return R;
}

// Value of lane (first lane of this lane's aligned group of TPD lanes) + q, for q < TPD: DPP
// quad permutes (one VALU, no LDS) for groups of up to 4 lanes, ds_bpermute otherwise.
template <uint32_t TPD>
__device__ __forceinline__ uint32_t group_lane(uint32_t x, uint32_t q) {
    if constexpr (TPD == 1) {
        return x;
    } else if constexpr (TPD == 2) {
        // quad_perm (0,0,2,2) / (1,1,3,3)
        return q == 0 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false)
                      : (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xF, 0xF, false);
    } else if constexpr (TPD == 4) {
        switch (q) {
            case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, false);
            case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x55, 0xF, 0xF, false);
            case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xAA, 0xF, 0xF, false);
            default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xFF, 0xF, 0xF, false);
        }
    } else {
        return (uint32_t)__shfl((int)x, (int)((lane_id() & ~(TPD - 1u)) + q));
    }
}

// Exclusive prefix (pre) of x over the lanes of this lane's aligned group of TPD lanes below it
// (sub = lane % TPD) and the group's total. Small groups: one group_lane per member; groups of
// 16..64 lanes: the DPP row scan of wave_incl_scan cut to the group, plus one bpermute for the
// total. Every lane of the wave must call it.
template <uint32_t TPD>
__device__ __forceinline__ void group_scan(uint32_t x, uint32_t sub, uint32_t &pre, uint32_t &tot) {
    if constexpr (TPD <= 8) {
        pre = 0;
        tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < TPD; ++q) {
            const uint32_t y = group_lane<TPD>(x, q);
            if (q < sub) pre += y;
            tot += y;
        }
    } else {
        static_assert(TPD == 16 || TPD == 32 || TPD == 64, "groups of 16, 32 or 64 lanes");
        uint32_t v = x;
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
        if constexpr (TPD >= 32)
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
        if constexpr (TPD == 64)
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
        pre = v - x;
        tot = (uint32_t)__shfl((int)v, (int)((lane_id() & ~(TPD - 1u)) + TPD - 1u));
    }
}

// Mask (lo, hi halves) of the lanes of this wave whose BITS-bit digit equals this lane's:
// AND over bits b of (ballot(bit b) XNOR my bit b), one v_bitop3 per half per bit
// (truth table 0x90 = a & ~(b ^ c) with a = mask, b = ballot half, c = my bit as 0 / ~0).
template <int BITS>
__device__ __forceinline__ void peer_mask(uint32_t d, uint32_t &mlo, uint32_t &mhi) {
    mlo = ~0u;
    mhi = ~0u;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        int s = __builtin_amdgcn_sbfe((int)d, b, 1);
        asm volatile("" : "+v"(s));  // keep s opaque: the ballot then compares s itself (1 VALU)
        const uint64_t bal = __ballot(s);
        mlo = __builtin_amdgcn_bitop3_b32(mlo, (uint32_t)bal, (uint32_t)s, 0x90);
        mhi = __builtin_amdgcn_bitop3_b32(mhi, (uint32_t)(bal >> 32), (uint32_t)s, 0x90);
    }
}

// Per-tile check of the kRankAtomic premise (the reference checks every sort,
// Parallel7.cu:679-687). The line and pairs kernels and rs_scatter run it on the first slot of a full tile
// (every kRankCheckEvery-th tile of a chunk): each lane's rank r from the lane-ordered returning adds must
// be base + (#lower lanes with its digit), with ONE base for all lanes of a digit. The lanes of a digit
// come from BITS ballots (peer_mask), the base of the digit's first lane from one ds_bpermute. A change of
// the lane order would permute the ranks among a digit's lanes -- the same keys in a wrong order, an
// unstable sort that no checksum of the keys can see -- and duplicated ranks (lost keys) fail the same
// test. Returns 1 where it failed. fault != 0 (test hook rsort_inject_rank_fault, ScatterArgs::rank_fault):
// the first two lanes of every digit swap their ranks first, as a broken lane order would. ~40 VALU and
// one bpermute per wave and checked tile; every lane of the wave must take part (full tiles only).
template <int BITS>
__device__ __forceinline__ uint32_t rank_check(uint32_t d, uint32_t &r, uint32_t fault) {
    uint32_t mlo, mhi;
    peer_mask<BITS>(d, mlo, mhi);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
    if (fault != 0u) {
        const uint32_t peers = (uint32_t)__builtin_popcount(mlo) + (uint32_t)__builtin_popcount(mhi);
        if (peers >= 2u && below < 2u) r = below == 0u ? r + 1u : r - 1u;
    }
    const uint32_t b = r - below;
    const uint32_t first = mlo != 0u ? (uint32_t)__builtin_ctz(mlo) : 32u + (uint32_t)__builtin_ctz(mhi);
    return (uint32_t)__shfl((int)b, (int)first) != b ? 1u : 0u;
}

// Tiles between rank checks in a chunk (a power of 2): the check on every tile cost C3 / C4 ~1 % (same-box
// A/B); every 8th, starting with each chunk's first tile, checks 8-64 tiles per chunk and pass at C3 / C4.
constexpr uint32_t kRankCheckEvery = 8;

// End of a scatter workgroup: a wave any of whose lanes saw a failed rank_check sets kCheckRankOrder in the
// sort's check word (rsort_plan_check; the host entries return RSORT_ERR_CHECK). Every lane must call it.
__device__ __forceinline__ void report_order(uint32_t *check, uint32_t bad) {
    if (check != nullptr && __ballot(bad != 0u) != 0ull && lane_id() == 0) atomicOr(check, kCheckRankOrder);
}

// Inclusive wave64 scan with DPP row shifts + row broadcasts (no LDS, no bpermute):
// row_shr:1,2,4,8 scan each row of 16 lanes, row_bcast:15 / row_bcast:31 carry row totals.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Exclusive scan of one value per thread across the workgroup. All threads must call it.
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_ws, uint32_t &total) {
    constexpr int W = THREADS / kWave;
    const uint32_t w = threadIdx.x / kWave;
    const uint32_t inc = wave_incl_scan(v);
    if (lane_id() == kWave - 1) s_ws[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const uint32_t s = s_ws[i];
        pre += ((uint32_t)i < w) ? s : 0u;
        tot += s;
    }
    total = tot;
    __syncthreads();
    return pre + inc - v;
}

// Same, with one barrier: the caller guarantees another barrier before s_ws is written again.
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan1(uint32_t v, uint32_t *s_ws, uint32_t &total) {
    constexpr int W = THREADS / kWave;
    const uint32_t w = threadIdx.x / kWave;
    const uint32_t inc = wave_incl_scan(v);
    if (lane_id() == kWave - 1) s_ws[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const uint32_t s = s_ws[i];
        pre += ((uint32_t)i < w) ? s : 0u;
        tot += s;
    }
    total = tot;
    return pre + inc - v;
}

// Split mode (partitions): the splitters are read from the kernel arguments once, at construction, into
// wave-uniform registers, padded to 2^BITS - 1 with ~0u; cmp() is then a fixed run of compares and adds
// clamped to nsplit (a padded ~0u only counts for key ~0u, where every real splitter counts too). An
// early-exit loop over nsplit splitters instead compiled to a scalar loop re-reading the kernel arguments
// for every key (16 buckets: 2.08 ms to count 2^30 keys, dev/LOG.md round 6).
//
// Prefix table (the partition's histogram and line scatter with > 8 buckets, kSplitTabWords of LDS): a
// wave64 compare costs 4 cycles per SIMD, so 15 splitters took ~34 VALU cycles x 4 per key -- more than
// the key's whole HBM time. The table holds, per 11-bit key prefix, the digit of the prefix's smallest
// key (low 5 bits) and how many splitters lie inside the prefix's range (high 3 bits, mostly 0; 7: 7 or
// more, up to the last); a key's digit is the entry's low bits plus the splitters from there on that it
// reaches, compared against an LDS copy of the splitters after the entries.
constexpr uint32_t kSplitTabBits = 11;
constexpr uint32_t kSplitTabWords = (1u << kSplitTabBits) / 4 + 32;  // 2 KB of entries + 32 splitters
template <int BITS, int DMODE>
struct Digit {
    // only 2^BITS - 1 splitters can exist (the host sizes BITS to the bucket count)
    static constexpr int NS =
        DMODE == kDigitShift ? 1 : (((1 << BITS) - 1) < kMaxSplitters ? ((1 << BITS) - 1) : kMaxSplitters);
    uint32_t shift;
    uint32_t nsplit;
    uint32_t sp[NS];
    uint32_t *tab;  // split mode: the prefix table in LDS (fill_table), or nullptr: compares only
    __device__ __forceinline__ Digit(uint32_t shift_, uint32_t nsplit_, const uint32_t *split,
                                     uint32_t *tab_ = nullptr)
        : shift(shift_), nsplit(nsplit_), tab(tab_) {
        if constexpr (DMODE == kDigitSplit) {
#pragma unroll
            for (int i = 0; i < NS; ++i) sp[i] = (uint32_t)i < nsplit_ ? split[i] : ~0u;
        } else {
            sp[0] = 0;
        }
    }
    __device__ __forceinline__ uint32_t cmp(uint32_t key) const {
        uint32_t d = 0;
#pragma unroll
        for (int i = 0; i < NS; ++i) d += key >= sp[i] ? 1u : 0u;
        return d < nsplit ? d : nsplit;
    }
    // the prefix table, by the workgroup's `threads` threads (the caller synchronises before use)
    __device__ __forceinline__ void fill_table(uint32_t t, uint32_t threads) const {
        if constexpr (DMODE == kDigitSplit) {
            constexpr uint32_t SH = 32 - kSplitTabBits;
            for (uint32_t wd = t; wd < (1u << kSplitTabBits) / 4; wd += threads) {
                uint32_t v = 0;
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) {
                    const uint32_t p = wd * 4 + b;
                    const uint32_t lo = cmp(p << SH), hi = cmp((p << SH) | ((1u << SH) - 1u));
                    v |= (lo | min(hi - lo, 7u) << 5) << (8 * b);
                }
                tab[32 + wd] = v;
            }
#pragma unroll
            for (int i = 0; i < 32; ++i)  // (constant indices: sp stays in registers)
                if (t == (uint32_t)i) tab[i] = i < NS ? sp[i < NS ? i : 0] : ~0u;
        }
    }
    __device__ __forceinline__ uint32_t operator()(uint32_t key) const {
        if constexpr (DMODE == kDigitShift) {
            return (key >> shift) & ((1u << BITS) - 1u);
        } else {
            if (tab == nullptr) return cmp(key);
            const uint32_t e = reinterpret_cast<const uint8_t *>(tab + 32)[key >> (32 - kSplitTabBits)];
            uint32_t d = e & 31u;
            const uint32_t span = e >> 5, end = span == 7u ? nsplit : d + span;
            while (d < end && key >= tab[d]) ++d;  // (non-decreasing splitters: the first one above the key)
            return d;
        }
    }
};

// ------------------------------------------------------------------------------ histogram
// Reference: histogramKernel (Parallel7.cu:318-343) + transpose (P7:361-392, :596).
// SUB: each per-wave copy is split into SUB interleaved sub-counters (lane % SUB picks one), so
// lanes of one instruction that share a digit -- the common digits of skewed keys -- hit SUB
// different addresses instead of serialising on one.
//
// Digit-group chunks (k = 8, 2^8 chunks; rsort_capi.cpp sort_planned). After pass p the keys are
// ordered by digit p, so pass p + 1 may take digit p's groups as its chunks: group g's counts of
// digit p + 1 are the joint counts J[g][.] of (digit p, digit p + 1), which pass p counts here
// (JOINT) while it reads the keys anyway. Pass p + 1's histogram launch then only copies them
// (a.bounds[0] == kGroupsWhole, set by rs_joint_bounds when the groups are balanced enough to be
// chunks), or counts just the pieces of the groups its chunks cut (kGroupsCut).
// Joint counts live in LDS as 2^16 16-bit counters, two per word, in rows of 128 + 1 words
// (the pad makes the column sweep of the final add bank-conflict free); a counter that reaches
// 2^15 moves 2^15 to its row's spill word and to the global count (the returning add tells).
template <int THREADS>
__device__ __forceinline__ void hist_joint_body(const HistArgs &a, uint32_t *s_j, uint32_t c,
                                                uint32_t sub, uint32_t S) {
    constexpr uint32_t R = kJointBins;
    constexpr uint32_t RS = R / 2 + 1;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t *s_sp = s_j + R * RS;
    // HistArgs::rows: the spilled pairs (each spill moved 2^15 of the pair's count out of LDS) and the
    // largest digit count of the chunk
    __shared__ uint32_t s_spl[kMaxRowSpills];
    __shared__ uint32_t s_nsp, s_rmax;
    __shared__ uint32_t s_nz[R], s_ne[R];  // per row: nonzero entries, and one of them
    const uint32_t t = threadIdx.x;
    RS_WG_T0
    for (uint32_t i = t; i < R * RS + R; i += THREADS) s_j[i] = 0;
    if (t == 0) {
        s_nsp = 0u;
        s_rmax = 0u;
    }
    for (uint32_t i = t; i < R; i += THREADS) s_nz[i] = 0u;
    __syncthreads();
    const uint32_t s0 = a.shift, s1 = a.shift + kJointBits;
    // add inc (<= 64) to the 16-bit counter of pair (d, e); the add that takes it to 2^15 moves 2^15
    // to the row's spill word and to the global count (the counter stays below 2^15 + 64)
    auto add_pair = [&](uint32_t d, uint32_t e, uint32_t inc) {
        const uint32_t wi = d * RS + (e >> 1), sh = (e & 1u) << 4;
        const uint32_t before = (atomicAdd(&s_j[wi], inc << sh) >> sh) & 0xFFFFu;
        if (before + inc >= 0x8000u && before < 0x8000u) {
            atomicSub(&s_j[wi], 0x8000u << sh);
            atomicAdd(&s_sp[d], 0x8000u);
            atomicAdd(&a.joint[e * R + d], 0x8000u);
            if (a.rows != nullptr) {
                const uint32_t k = atomicAdd(&s_nsp, 1u);
                if (k < kMaxRowSpills) s_spl[k] = d * R + e;
            }
        }
    };
    auto add = [&](uint32_t x) { add_pair((x >> s0) & (R - 1u), (x >> s1) & (R - 1u), 1u); };
    // Clustered input (runs of equal keys: sorted or duplicate-heavy data, and every pass after a cut
    // plan, whose input holds the copies of a key contiguously) sends many lanes of one instruction to
    // one counter, where returning adds serialise (all-equal keys: 64 lanes, ~128 cycles per
    // instruction). There each component of a batch of quads (lane l holds keys 4l .. 4l + 3, so lanes
    // l and l + 1 hold keys 4 apart) is added by runs: lanes holding the same pair as the lane below
    // continue its run, and only a run's first lane adds (the run's length, one returning add).
    // Uniform keys take the plain adds after one test per batch (the first quad's first and last keys).
    auto pair_of = [&](uint32_t x) { return (x >> s0) & 0xFFu | ((x >> s1) & 0xFFu) << 8; };
    auto add_run = [&](uint32_t x) {
        const uint32_t pr = pair_of(x);
        // the lane below's pair (wave_shr:1; lane 0 gets ~pr: it starts a run)
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)~pr, (int)pr, 0x138, 0xF, 0xF, false);
        const bool cont = prev == pr;
        const uint64_t brk = __ballot(!cont) | ~__ballot(true);  // (inactive lanes end every run)
        if (!cont) {
            const uint64_t above = brk & ~((2ull << lane_id()) - 1ull);
            const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : 64u;
            add_pair(pr & 0xFFu, pr >> 8, end - lane_id());
        }
    };
    const uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    const uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    const uint64_t part = (((cend > cbeg ? cend - cbeg : 0) + S - 1) / S + 3) & ~(uint64_t)3;
    const uint64_t beg = min(cbeg + sub * part, cend);
    const uint64_t end = min(beg + part, cend);
    uint64_t tail = beg;
    if (a.vec) {
        const u32x4 *p = reinterpret_cast<const u32x4 *>(a.keys + beg);
        const uint32_t nvec = (uint32_t)((end - beg) / 4);
        constexpr int U = 4;
        for (uint32_t v0 = t; v0 < nvec; v0 += THREADS * U) {
            u32x4 q[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t v = v0 + u * THREADS;
                ok[u] = v < nvec;
                q[u] = ok[u] ? __builtin_nontemporal_load(p + v) : u32x4{0, 0, 0, 0};
            }
            // one clustering test per batch: >= 8 lanes whose first quad starts and ends with one pair
            if (wave_count(__ballot(ok[0] && pair_of(q[0].x) == pair_of(q[0].w))) < 8) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (ok[u]) {
                        add(q[u].x);
                        add(q[u].y);
                        add(q[u].z);
                        add(q[u].w);
                    }
                }
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (ok[u]) {
                        add_run(q[u].x);
                        add_run(q[u].y);
                        add_run(q[u].z);
                        add_run(q[u].w);
                    }
                }
            }
        }
        tail = beg + (uint64_t)nvec * 4;
    }
    for (uint64_t i = tail + t; i < end; i += THREADS) add(a.keys[i]);
    __syncthreads();
    // this chunk's digit counts: row sums plus the row's spill
    for (uint32_t d = t; d < R; d += THREADS) {
        uint32_t s = s_sp[d];
        for (uint32_t j = 0; j < R / 2; ++j) {
            const uint32_t x = s_j[d * RS + j];
            s += (x & 0xFFFFu) + (x >> 16);
        }
        if (S == 1) a.table[(uint64_t)d * a.num_chunks + c] = s;
        else if (s) atomicAdd(&a.table[(uint64_t)d * a.num_chunks + c], s);
        if (a.rows != nullptr) atomicMax(&s_rmax, s);
    }
    // joint counts -> global [e][d] (consecutive lanes: consecutive d, one contiguous 256-B add)
    for (uint32_t item = t; item < R * R; item += THREADS) {
        const uint32_t e = item / R, d = item % R;
        const uint32_t v = (s_j[d * RS + (e >> 1)] >> ((e & 1u) << 4)) & 0xFFFFu;
        if (v) atomicAdd(&a.joint[item], v);
    }
    if (a.rows != nullptr && S == 1) {
        // this chunk's joint counts as rows [digit][next digit] for a cut plan's pieces (HistArgs::rows):
        // when the previous odd pass cut its groups (skewed keys: the next one likely cuts too) or a
        // digit holds more than twice its share of the chunk; uniform chunks write nothing
        __syncthreads();
        const bool after_cut = a.joint_enable != nullptr && *a.joint_enable == kGroupsCut;
        if ((after_cut || (uint64_t)s_rmax * R > 2 * (cend - cbeg)) && s_nsp <= kMaxRowSpills) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            uint32_t *rw = a.rows + (uint64_t)c * R * R;
            static_assert(THREADS % kWave == 0 && (R / 2) % kWave == 0, "a wave's items lie in one row");
            for (uint32_t item = t; item < R * (R / 2); item += THREADS) {
                const uint32_t d = item / (R / 2), j = item % (R / 2);
                const uint32_t x = s_j[d * RS + j];
                *reinterpret_cast<u32x2 *>(rw + d * R + 2 * j) = u32x2{x & 0xFFFFu, x >> 16};
                // the row's nonzero entries, one LDS add per wave (its 64 items share the row)
                const uint64_t blo = __ballot((x & 0xFFFFu) != 0u), bhi = __ballot((x >> 16) != 0u);
                const uint32_t nz = wave_count(blo) + wave_count(bhi);
                if (nz != 0u && lane_id() == 0) {
                    const uint32_t j0 = j;  // (lane 0's item: the wave's first)
                    atomicAdd(&s_nz[d], nz);
                    s_ne[d] = blo ? 2 * (j0 + (uint32_t)__builtin_ctzll(blo)) : 2 * (j0 + (uint32_t)__builtin_ctzll(bhi)) + 1;
                }
            }
            // the spilled pairs: stored again with their spilled 2^15s on top, after every wave's row
            // stores have reached the L2 (same workgroup, same L2: the later store wins; no release
            // fence -- an agent-scope one writes the whole L2 back)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            for (uint32_t i = t; i < s_nsp; i += THREADS) {
                const uint32_t pr = s_spl[i], d = pr / R, e = pr % R;
                uint32_t k = 0;
                bool first = true;
                for (uint32_t x = 0; x < s_nsp; ++x) {
                    k += s_spl[x] == pr ? 1u : 0u;
                    first = first && !(x < i && s_spl[x] == pr);
                }
                const uint32_t res = (s_j[d * RS + (e >> 1)] >> ((e & 1u) << 4)) & 0xFFFFu;
                rw[pr] = res + 0x8000u * k;
                if (first && res == 0u) {  // (a nonzero entry the row loop saw as zero)
                    atomicAdd(&s_nz[d], 1u);
                    s_ne[d] = e;
                }
            }
            __syncthreads();
            // per row: its one next digit when it has exactly one (a piece end inside this chunk's part
            // of that group then needs no key read, rs_joint_bounds), else ~0
            for (uint32_t d = t; d < R; d += THREADS) a.rows[kRowsWords + (uint64_t)c * R + d] = s_nz[d] == 1u ? s_ne[d] : ~0u;
            if (t == 0) atomicAdd(a.rows_cnt, 1u);
        }
    }
    RS_WG_TH1;
}

// Partitions into <= 8 buckets (split digits, BITS <= 3): per lane, in registers, the count of keys >=
// each splitter -- 7 compares and adds per key -- and no LDS add per key (with two or four buckets 32 or
// 16 lanes of every add met on one LDS counter). Bucket b holds ge[b - 1] - ge[b] keys (non-decreasing
// splitters; ge[-1] = every key counted, ge[nsplit] = 0). More buckets (BITS = 4) count their digits
// from the prefix table (Digit::fill_table) into the LDS counters like shift digits.
template <int BITS, int THREADS, int NT>
__device__ __forceinline__ void hist_split_body(const HistArgs &a, uint32_t *s_h, uint32_t c, uint32_t sub,
                                                uint32_t S) {
    typedef Digit<BITS, kDigitSplit> D;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr int NS = D::NS;
    constexpr uint32_t R = 1u << BITS;
    const uint32_t t = threadIdx.x;
    const D dig{a.shift, a.nsplit, a.splitters};
    uint32_t ge[NS + 1];  // ge[NS]: the keys counted
#pragma unroll
    for (int i = 0; i <= NS; ++i) ge[i] = 0u;
    auto cnt = [&](uint32_t x) {
#pragma unroll
        for (int i = 0; i < NS; ++i) ge[i] += x >= dig.sp[i] ? 1u : 0u;
        ge[NS] += 1u;
    };
    const uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    const uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    const uint64_t part = (((cend > cbeg ? cend - cbeg : 0) + S - 1) / S + 3) & ~(uint64_t)3;
    const uint64_t beg = min(cbeg + sub * part, cend);
    const uint64_t end = min(beg + part, cend);
    uint64_t tail = beg;
    if (a.vec) {
        const uint64_t vb = min((beg + 3) & ~(uint64_t)3, end);
        for (uint64_t i = beg + t; i < vb; i += THREADS) cnt(a.keys[i]);
        const u32x4 *p = reinterpret_cast<const u32x4 *>(a.keys + vb);
        const uint32_t nvec = (uint32_t)((end - vb) / 4);
        constexpr int U = 4;
        for (uint32_t v0 = t; v0 < nvec; v0 += THREADS * U) {
            u32x4 q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t v = v0 + u * THREADS;
                q[u] = v < nvec ? (NT ? __builtin_nontemporal_load(p + v) : p[v]) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (v0 + u * THREADS < nvec) {
                    cnt(q[u].x);
                    cnt(q[u].y);
                    cnt(q[u].z);
                    cnt(q[u].w);
                }
            }
        }
        tail = vb + (uint64_t)nvec * 4;
    }
    for (uint64_t i = tail + t; i < end; i += THREADS) cnt(a.keys[i]);
    // wave sums -> LDS -> bucket counts
    const uint32_t w = t / kWave;
#pragma unroll
    for (int i = 0; i <= NS; ++i) {
        uint32_t v = ge[i];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane_id() == 0) s_h[w * (NS + 1) + i] = v;
    }
    __syncthreads();
    auto total = [&](uint32_t j) {
        uint32_t s = 0;
#pragma unroll
        for (int x = 0; x < THREADS / kWave; ++x) s += s_h[x * (NS + 1) + j];
        return s;
    };
    const uint32_t ns = a.nsplit;
    for (uint32_t d = t; d < R; d += THREADS) {
        const uint32_t hi = d == 0u ? total(NS) : (d <= ns ? total(d - 1u) : 0u);
        const uint32_t v = d < ns ? hi - total(d) : hi;
        if (S == 1) a.table[(uint64_t)d * a.num_chunks + c] = v;
        else if (v) atomicAdd(&a.table[(uint64_t)d * a.num_chunks + c], v);
    }
}

template <int BITS, int THREADS, int DMODE, int NT = 0, int SUB = 1, bool JOINT = false>
__global__ __launch_bounds__(THREADS) void rs_histogram(HistArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int HW = (R * W <= 4096) ? W : 1;  // per-wave private copies when they fit (<= 16 KB)
    constexpr int SB = HW > 1 ? SUB : 1;
    constexpr uint32_t PLAIN = HW * R * SB;
    constexpr uint32_t JW = kJointBins * (kJointBins / 2 + 1) + kJointBins;
    static_assert(!JOINT || (BITS == kJointBits && DMODE == kDigitShift), "joint counts: k = 8 digits");
    __shared__ __attribute__((aligned(16))) uint32_t s_h[(JOINT && JW > PLAIN) ? JW : PLAIN];

    const uint32_t t = threadIdx.x;
    const uint32_t S = a.split;
    const uint32_t c = blockIdx.x / S;
    const uint32_t sub = blockIdx.x % S;
    if (a.bounds != nullptr && a.bounds[0] == kGroupsWhole) {
        // digit-group chunks: this pass's table is the previous pass's joint counts
        const uint64_t m = (uint64_t)R * a.num_chunks;
        for (uint64_t i = (uint64_t)blockIdx.x * THREADS + t; i < m; i += (uint64_t)gridDim.x * THREADS) {
            a.table[i] = a.copy_src[i];
            a.copy_src[i] = 0u;  // the next joint count adds into it: no memset launch
        }
        return;
    }
    // pass 0 of a sort (HistArgs::done): clear the check words on the way (before any scatter runs)
    if (a.done != nullptr && blockIdx.x == 0 && t == 0) {
        a.done[0] = 0u;
        a.done[kDoneErr] = 0u;
    }
    if constexpr (JOINT) {
        if (a.joint_enable == nullptr || *a.joint_enable != kGroupsFixed) {
            hist_joint_body<THREADS>(a, s_h, c, sub, S);
            return;
        }
    }
    // raw-table plans (HistArgs::zero): clear the next table on the way
    for (uint64_t i = (uint64_t)blockIdx.x * THREADS + t; i < a.zero_n; i += (uint64_t)gridDim.x * THREADS)
        a.zero[i] = 0u;
    constexpr bool SPLIT_TAB = DMODE == kDigitSplit && BITS > 3;
    if constexpr (DMODE == kDigitSplit && !SPLIT_TAB) {
        static_assert(W * (Digit<BITS, DMODE>::NS + 1) <= (int)PLAIN, "the wave sums fit s_h");
        hist_split_body<BITS, THREADS, NT>(a, s_h, c, sub, S);
        return;
    }
    __shared__ uint32_t s_stab[SPLIT_TAB ? kSplitTabWords : 1];
    for (uint32_t i = t; i < HW * R * SB; i += THREADS) s_h[i] = 0;
    const Digit<BITS, DMODE> dig{a.shift, a.nsplit, a.splitters, SPLIT_TAB ? s_stab : nullptr};
    if constexpr (SPLIT_TAB) dig.fill_table(t, THREADS);
    __syncthreads();

    // counter of digit d: my[d * SB] (this lane's sub-counter)
    uint32_t *my = s_h + (HW > 1 ? (t / kWave) * R * SB : 0) + (SB > 1 ? lane_id() % SB : 0);
    // keys [beg, end) into the LDS counters (16-B loads from the first 16-B aligned key on)
    auto count_range = [&](uint64_t beg, uint64_t end) {
        uint64_t tail = beg;
        if (a.vec) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const uint64_t vb = min((beg + 3) & ~(uint64_t)3, end);
            for (uint64_t i = beg + t; i < vb; i += THREADS) atomicAdd(&my[dig(a.keys[i]) * SB], 1u);
            const u32x4 *p = reinterpret_cast<const u32x4 *>(a.keys + vb);
            const uint32_t nvec = (uint32_t)((end - vb) / 4);
            constexpr int U = 4;
            for (uint32_t v0 = t; v0 < nvec; v0 += THREADS * U) {
                u32x4 q[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t v = v0 + u * THREADS;
                    // NT: non-temporal loads (the keys are read once per pass)
                    q[u] = v < nvec ? (NT ? __builtin_nontemporal_load(p + v) : p[v]) : u32x4{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (v0 + u * THREADS < nvec) {
                        const uint32_t dx = dig(q[u].x), dy = dig(q[u].y), dz = dig(q[u].z), dw = dig(q[u].w);
                        const bool same4 = dx == dy && dy == dz && dz == dw;
                        if (wave_count(__ballot(same4)) >= 32) {
                            // clustered input (runs of equal keys, e.g. duplicates after a pass): one
                            // add of 4 per lane, lanes sharing the common digits together
                            if (same4) {
                                // (count_add's aggregating lane adds for all: any sub-counter will do)
                                if constexpr (SB > 1) count_add(my, dx * SB, 4u);
                                else count_add(my, dx, 4u);
                            } else {
                                atomicAdd(&my[dx * SB], 1u);
                                atomicAdd(&my[dy * SB], 1u);
                                atomicAdd(&my[dz * SB], 1u);
                                atomicAdd(&my[dw * SB], 1u);
                            }
                        } else {
                            atomicAdd(&my[dx * SB], 1u);
                            atomicAdd(&my[dy * SB], 1u);
                            atomicAdd(&my[dz * SB], 1u);
                            atomicAdd(&my[dw * SB], 1u);
                        }
                    }
                }
            }
            tail = vb + (uint64_t)nvec * 4;
        }
        for (uint64_t i = tail + t; i < end; i += THREADS) atomicAdd(&my[dig(a.keys[i]) * SB], 1u);
    };
    // this pass's counts of one digit (all copies), the counters cleared for the next range
    auto take = [&](uint32_t d) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < HW; ++w)
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                s += s_h[(w * R + d) * SB + u];
                s_h[(w * R + d) * SB + u] = 0;
            }
        return s;
    };
    if constexpr (BITS == kJointBits && DMODE == kDigitShift) {
        if (a.bounds != nullptr && a.bounds[0] == kGroupsCut) {
            // cut plan (rs_joint_bounds): the workgroups split the counted pieces' keys evenly; each
            // counts its share of every piece it meets, adds the counts into the piece's row and
            // takes them from its group's derived row (zeroed; the scan adds the joint counts)
            __shared__ uint32_t s_first;
            const uint32_t np = a.plan[0], K = a.plan[1], nr = a.plan[2];
            // row tasks (rs_joint_bounds with HistArgs::rows): task i by workgroup i mod the grid -- the
            // piece's whole previous chunks, their rows summed (THREADS / R threads per next digit)
            if (nr > 0) {
                // 64 threads per row (16-B loads), NQ rows at a time, 4 loads in flight per thread; the
                // NQ partial rows summed through s_h (zero again before the keys are counted into it)
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                constexpr uint32_t NQ = THREADS / kWave;
                static_assert(R == 4 * kWave && NQ * R <= PLAIN, "a row is one wave of quads");
                const uint32_t q = t / kWave, e4 = lane_id();
                for (uint32_t i = blockIdx.x; i < nr; i += gridDim.x) {
                    const uint32_t *rt = a.plan + kPlanRows + 4 * i;
                    const uint32_t sl = rt[0], g = rt[1], c0 = rt[2], c1 = rt[3];
                    if (g & kRowDirect) {  // (uniform: the whole workgroup skips the row sum)
                        if (t == 0) {
                            atomicAdd(&a.pcounts[(sl & (kPieceNeg - 1u)) * R + (g & (R - 1u))], c0);
                            atomicSub(&a.pcounts[(sl >> 16) * R + (g & (R - 1u))], c0);
                        }
                        continue;
                    }
                    const u32x4 *rows4 = reinterpret_cast<const u32x4 *>(a.rows + (uint64_t)g * R) + e4;
                    constexpr uint64_t CS = (uint64_t)R * R / 4;  // quads per chunk
                    u32x4 acc = {0u, 0u, 0u, 0u};
                    uint32_t cc = c0 + q;
                    for (; cc + 3 * NQ < c1; cc += 4 * NQ) {
                        const u32x4 v0 = rows4[cc * CS], v1 = rows4[(cc + NQ) * CS], v2 = rows4[(cc + 2 * NQ) * CS],
                                    v3 = rows4[(cc + 3 * NQ) * CS];
                        acc += v0 + v1 + v2 + v3;
                    }
                    for (; cc < c1; cc += NQ) acc += rows4[cc * CS];
                    *reinterpret_cast<u32x4 *>(&s_h[q * R + 4 * e4]) = acc;
                    __syncthreads();
                    if (t < R) {
                        uint32_t v = 0;
#pragma unroll
                        for (uint32_t x = 0; x < NQ; ++x) v += s_h[x * R + t];
                        if (v) {
                            atomicAdd(&a.pcounts[(sl & (kPieceNeg - 1u)) * R + t], v);
                            atomicSub(&a.pcounts[(sl >> 16) * R + t], v);  // the group's derived segment
                        }
                    }
                    __syncthreads();
                }
                for (uint32_t i = t; i < NQ * R; i += THREADS) s_h[i] = 0;
                __syncthreads();
            }
            const uint64_t s0 = (uint64_t)K * blockIdx.x / gridDim.x, s1 = (uint64_t)K * (blockIdx.x + 1) / gridDim.x;
            if (s0 >= s1) return;
            if (t < np) {
                const uint32_t off = a.plan[kPlanPieces + 4 * t + 3];
                const uint32_t nxt = t + 1 < np ? a.plan[kPlanPieces + 4 * t + 7] : K;
                if (off <= s0 && s0 < nxt) s_first = t;
            }
            __syncthreads();
            for (uint32_t i = s_first; i < np; ++i) {
                const uint32_t ps = a.plan[kPlanPieces + 4 * i], pe = a.plan[kPlanPieces + 4 * i + 1];
                const uint32_t sl = a.plan[kPlanPieces + 4 * i + 2], off = a.plan[kPlanPieces + 4 * i + 3];
                const uint32_t slot = sl & (kPieceNeg - 1u), dslot = sl >> 16;
                const bool neg = (sl & kPieceNeg) != 0u;  // (a range the piece does NOT hold, rs_joint_bounds)
                if (off >= s1) break;
                const uint64_t lo = max(s0, (uint64_t)off), hi = min(s1, (uint64_t)off + (pe - ps));
                count_range(ps + (lo - off), ps + (hi - off));
                __syncthreads();
                for (uint32_t d = t; d < R; d += THREADS) {
                    const uint32_t v = take(d);
                    if (v) {
                        atomicAdd(&a.pcounts[slot * R + d], neg ? 0u - v : v);
                        atomicSub(&a.pcounts[dslot * R + d], neg ? 0u - v : v);  // the group's derived segment
                    }
                }
                __syncthreads();
            }
            return;
        }
    }
    // this workgroup's part of chunk c: S parts of a multiple of 4 keys (16-B aligned starts)
    const uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    const uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    const uint64_t part = (((cend > cbeg ? cend - cbeg : 0) + S - 1) / S + 3) & ~(uint64_t)3;
    const uint64_t beg = min(cbeg + sub * part, cend);
    const uint64_t end = min(beg + part, cend);
    count_range(beg, end);
    __syncthreads();
    for (uint32_t d = t; d < R; d += THREADS) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < HW; ++w)
#pragma unroll
            for (int u = 0; u < SB; ++u) s += s_h[(w * R + d) * SB + u];
        if (S == 1) a.table[(uint64_t)d * a.num_chunks + c] = s;
        else if (s) atomicAdd(&a.table[(uint64_t)d * a.num_chunks + c], s);
    }
}

// ------------------------------------------------------------------------------ table scan
// Exclusive scan of the column-major chunk x digit table, == the column-major scan of
// Baseline4.cu:127-138 / P7's transpose-scan-transpose. Two launches: segment sums, then
// each segment adds the sum of the segments before it (<= a few thousand values, read from
// L2) and scans itself.
__global__ __launch_bounds__(kScanThreads) void rs_scan_reduce(ScanArgs a) {
    __shared__ uint32_t s_ws[kScanThreads / kWave];
    // next-digit plans: clear the table the coming scatter counts into (read by the previous
    // pass's scatter, finished before this launch)
    for (uint64_t i = (uint64_t)blockIdx.x * kScanThreads + threadIdx.x; i < a.zero_n; i += (uint64_t)gridDim.x * kScanThreads)
        a.zero[i] = 0u;
    if (a.done != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        a.done[0] = 0u;         // the tail-scan counter
        a.done[kDoneErr] = 0u;  // its check word (tail_scan)
    }
    const uint64_t base = (uint64_t)blockIdx.x * kScanSegment + (uint64_t)threadIdx.x * kScanPerThread;
    uint32_t s = 0;
    if (a.group_flag != nullptr && *a.group_flag == kGroupsCut) {
        // Cut plan (rs_joint_bounds): this block assembles digit rows d = 16 b .. 16 b + 15 of the
        // R x R table [digit][chunk], thread c chunk c: its first group's part (the head, slot 2c),
        // the whole groups after it (a difference of the row's prefix sums over the groups) and its
        // last group's part (the tail, slot 2c + 1). A part that is a whole group is its joint
        // count, a counted piece its row, the derived one (a cut group's largest part) the group's
        // joint count plus its row (minus the group's counted pieces, rs_histogram).
        static_assert(kScanThreads == (int)kJointBins && kScanSegment == kScanPerThread * (int)kJointBins,
                      "one scan block = 16 rows of 256 chunks");
        constexpr uint32_t R = kJointBins, NW = kScanThreads / kWave, RP = R + 1;
        __shared__ uint32_t s_pj[kScanPerThread * RP];   // per row: prefix over groups, [0] = 0
        __shared__ uint32_t s_wt[kScanPerThread * NW];   // per row and wave: the wave's total
        const uint32_t c = threadIdx.x, w = c / kWave, d0 = blockIdx.x * kScanPerThread;
        const uint32_t dc = a.plan[kPlanDesc + c];
        const uint32_t gA = dc & 255u, gB = (dc >> 8) & 255u, hm = (dc >> 16) & 3u, tm = (dc >> 18) & 3u;
        const bool empty = (dc >> 20) != 0u;
        uint32_t jv[kScanPerThread], hv[kScanPerThread], tv[kScanPerThread];
#pragma unroll
        for (int i = 0; i < kScanPerThread; ++i) {
            jv[i] = a.joint[(d0 + i) * R + c];  // group c's count of digit d0 + i
            hv[i] = hm != kSegWhole ? a.pcounts[(2u * c) * R + d0 + i] : 0u;
            tv[i] = tm != kSegWhole ? a.pcounts[(2u * c + 1u) * R + d0 + i] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kScanPerThread; ++i) {
            jv[i] = wave_incl_scan(jv[i]);
            if (lane_id() == kWave - 1) s_wt[i * NW + w] = jv[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kScanPerThread; ++i) {
            uint32_t add = 0;
#pragma unroll
            for (uint32_t x = 0; x < NW; ++x) add += x < w ? s_wt[i * NW + x] : 0u;
            s_pj[i * RP + c + 1] = jv[i] + add;
        }
        if (c < kScanPerThread) s_pj[c * RP] = 0u;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kScanPerThread; ++i) {
            const uint32_t *pj = s_pj + i * RP;
            uint32_t v = 0;
            if (!empty) {
                const uint32_t ja = pj[gA + 1] - pj[gA];
                v = hm == kSegWhole ? ja : hv[i] + (hm == kSegDerived ? ja : 0u);
                if (gB != gA) {
                    const uint32_t jb = pj[gB + 1] - pj[gB];
                    v += (pj[gB] - pj[gA + 1]) + (tm == kSegWhole ? jb : tv[i] + (tm == kSegDerived ? jb : 0u));
                }
            }
            a.table[(d0 + i) * R + c] = v;
            s += v;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanPerThread; ++i) s += (base + i < a.m) ? a.table[base + i] : 0u;
    }
    uint32_t tot;
    block_excl_scan<kScanThreads>(s, s_ws, tot);
    if (threadIdx.x == 0) a.block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void rs_scan_down(ScanArgs a) {
    __shared__ uint32_t s_ws[kScanThreads / kWave];
    const uint32_t b = blockIdx.x;
    uint32_t pre = 0;
    for (uint32_t i = threadIdx.x; i < b; i += kScanThreads) pre += a.block_sums[i];
    uint32_t prefix;
    block_excl_scan<kScanThreads>(pre, s_ws, prefix);

    const uint64_t base = (uint64_t)b * kScanSegment + (uint64_t)threadIdx.x * kScanPerThread;
    if (a.group_flag != nullptr && *a.group_flag == kGroupsCut) {
        // the joint counts were read by the first launch: clear them for the next joint count
        // (the table is R x R, the joint counts' shape)
        for (int i = 0; i < kScanPerThread; ++i)
            if (base + i < a.m) a.joint[base + i] = 0u;
    }
    uint32_t v[kScanPerThread];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) {
        v[i] = (base + i < a.m) ? a.table[base + i] : 0u;
        s += v[i];
    }
    uint32_t tot;
    uint32_t run = prefix + block_excl_scan<kScanThreads>(s, s_ws, tot);
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) {
        if (base + i < a.m) a.table[base + i] = run;
        run += v[i];
    }
}

// The same exclusive scan as the tail of a kernel whose workgroups ADD into `table` with agent-scope
// atomics (m entries, a multiple of 4, 16-B aligned, < 4 GiB): every workgroup waits for its adds and
// bumps *done; the one whose bump comes last scans the table alone -- each wave a contiguous run
// of 64-quad blocks -- clears `zero` (m entries) and re-arms *done. Next-digit plans (k = 3, 4)
// scan every table after the first this way: one launch per pass instead of three (rs_scan_reduce
// + rs_scan_down, each ~5 us at C2, and their launch gaps).
// Visibility (MI355X_MICROARCH.md, inter-workgroup visibility, the table's first row): the payload
// is agent-scope atomics, performed beyond the XCD's L2 (they drop the line), every adding wave
// waits for them before its workgroup's one counter add, the last adder learns it from the value
// its add returns, and every load of the table is a 16-B sc1 load -- so neither a release fence
// per workgroup (a `buffer_wbl2` wrote back the default-policy output held in L2 and doubled the
// C2 pass time) nor an acquire fence (~1.7 us) is needed. The table counts every key of the pass
// exactly once, so its total must be `expect` (= n): the sum sweep checks that, and on a mismatch
// (a late or stale line -- never observed) the workgroup takes the agent-scope acquire fence and
// sums again; a second mismatch sets done[kDoneErr] -- so a visibility failure is repaired, or
// recorded where rsort_plan_check reads it. rsort.h is the contract: the stream-ordered device entries
// return RSORT_OK (they do not wait for the device) and a caller that must know asks rsort_plan_check;
// the host entries (rsort_u32*, which wait anyway) read the word and return RSORT_ERR_CHECK. Since round
// 4 this tail scan runs only under RSORT_NX_TAIL=1 (RSORT_LAB) or for plans with more chunks than the
// raw tables take (kRawTableMaxChunks); the default is raw_offsets, which checks the same total per
// workgroup. All threads must call it.
template <int THREADS>
__device__ void tail_scan(uint32_t *table, uint64_t m, uint32_t *zero, uint32_t *done, uint32_t *s_ws,
                          uint32_t *s_flag, uint32_t expect) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t t = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's adds have been performed
    __syncthreads();
    if (t == 0) *s_flag = atomicAdd(done, 1u) == gridDim.x - 1u ? 1u : 0u;
    __syncthreads();
    if (*s_flag == 0u) return;
    // descriptor from uniform inputs only (kernel arguments): base and size readfirstlane'd
    const uint64_t tb = (uint64_t)table;
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)tb), hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(tb >> 32));
    const uint32_t bytes = __builtin_amdgcn_readfirstlane((uint32_t)(m * 4));
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi32 << 32) | lo32), 0, bytes, 0x00020000);
    auto ld = [&](uint32_t quad) {  // 16-B sc1 load (aux 16): L2-served, never a stale L1 line
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, quad * 16u, 0, 16));
    };
    // wave w owns a run of whole 64-quad blocks, lane l quad l of each block: every load and store
    // instruction covers 1 KiB of consecutive table
    constexpr uint32_t NW = THREADS / kWave;
    const uint32_t w = t / kWave, l = lane_id();
    const uint32_t nq = (uint32_t)(m / 4);
    const uint32_t per = ((nq + NW - 1) / NW + kWave - 1) & ~(uint32_t)(kWave - 1);
    const uint32_t qb = min(nq, w * per), qe = min(nq, qb + per);
    constexpr uint32_t B = 8;  // blocks in flight per wave
    uint32_t run = 0, total = 0;
    for (int attempt = 0;; ++attempt) {
        uint32_t s = 0;
        for (uint32_t b0 = qb; b0 < qe; b0 += B * kWave) {
            u32x4 v[B];
#pragma unroll
            for (uint32_t u = 0; u < B; ++u) {
                const uint32_t qi = b0 + u * kWave + l;
                v[u] = qi < qe ? ld(qi) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (uint32_t u = 0; u < B; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
        }
        const uint32_t wsum = __builtin_amdgcn_readlane(wave_incl_scan(s), kWave - 1);
        if (l == 0) s_ws[w] = wsum;
        __syncthreads();
        run = 0;
        total = 0;
#pragma unroll
        for (uint32_t x = 0; x < NW; ++x) {
            const uint32_t y = s_ws[x];
            run += x < w ? y : 0u;
            total += y;
        }
        // (total is the same in every thread: the branches below are uniform)
        if (total == expect || attempt == 1) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __syncthreads();  // every wave has read s_ws before it is written again
    }
    if (total != expect && t == 0) atomicOr(&done[kDoneErr], kCheckTable);
    u32x4 *q = reinterpret_cast<u32x4 *>(table);
    for (uint32_t b0 = qb; b0 < qe; b0 += B * kWave) {
        u32x4 v[B];
#pragma unroll
        for (uint32_t u = 0; u < B; ++u) {
            const uint32_t qi = b0 + u * kWave + l;
            v[u] = qi < qe ? ld(qi) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (uint32_t u = 0; u < B; ++u) {
            const uint32_t qs = v[u].x + v[u].y + v[u].z + v[u].w;
            const uint32_t inc = wave_incl_scan(qs);
            u32x4 o;
            o.x = run + inc - qs;
            o.y = o.x + v[u].x;
            o.z = o.y + v[u].y;
            o.w = o.z + v[u].z;
            const uint32_t qi = b0 + u * kWave + l;
            if (qi < qe) q[qi] = o;
            run += __builtin_amdgcn_readlane(inc, kWave - 1);
        }
    }
    u32x4 *z = reinterpret_cast<u32x4 *>(zero);
    for (uint64_t i = t; i < m / 4; i += THREADS) z[i] = u32x4{0u, 0u, 0u, 0u};
    if (t == 0) *done = 0u;
}

// ------------------------------------------------------------------------------ group bounds
// One workgroup: group totals (column sums of the joint counts [next digit][group]), their
// exclusive scan = the groups' first key positions in the previous pass's output, and the next
// pass's chunk mode (kGroupsWhole / kGroupsCut / kGroupsFixed, rsort_internal.hpp) with its
// chunk starts; for kGroupsCut also the cut plan and zeroed piece rows.
// Cost-weighted cut plans (weighted != 0): the chunks of the next pass get equal estimated COST, not
// equal key counts. A group's keys arrive at the clustered scatter kernel in input order, so a
// chunk's per-key cost follows the group's next-digit distribution p (its joint column / size):
// measured on 2^28 Zipf keys, pass 1 (dev/wgtimes_lab.py, per-workgroup times of all 256 chunks, refit
// on the weighted plan's own chunks), us per Mkey = 427.1 + 685.9 * (sum p^2 - top^2) + 17.6 * top -
// 37.2 * top^2 (top = the largest p; the ranking aggregates the top digit, the other shared digits
// serialise), residual sd ~10 against a 400-518 spread with equal key counts. Weights are that rate
// over its constant, clamped to [0.8, 1.4].
__global__ __launch_bounds__(1024) void rs_joint_bounds(const uint32_t *joint, const uint32_t *enable,
                                                        uint32_t *bounds, uint32_t *plan, uint32_t *pcounts,
                                                        uint64_t n, uint64_t max_keys, uint32_t snap,
                                                        uint32_t weighted, const uint32_t *ctab,
                                                        uint32_t *rows_cnt, const uint32_t *rowone) {
    constexpr uint32_t R = kJointBins;
    constexpr uint32_t Q = 1024 / R;
    __shared__ uint32_t s_part[Q][R];
    __shared__ float s_sq[Q][R];                   // per part: sum of squared joint counts
    __shared__ uint32_t s_mx[Q][R];                // per part: the largest joint count
    __shared__ float s_w[R];                       // per group: cost per key (weighted plans)
    __shared__ uint32_t s_C[R + 1];                // per group: first weighted key (weighted plans)
    __shared__ uint32_t s_ws[1024 / kWave];
    __shared__ uint32_t s_max;
    __shared__ uint32_t s_b[R + 1];                // group starts
    __shared__ uint32_t s_B[R + 1];                // chunk starts (cut plan)
    __shared__ unsigned long long s_big[R];        // cut group: largest segment (size << 10 | slot)
    __shared__ uint32_t s_cf[R], s_cl[R];          // cut group: first and last chunk
    __shared__ uint32_t s_slot[R];                 // counted pieces' slots
    __shared__ uint32_t s_rows;                    // every chunk wrote its joint-count rows
    const uint32_t t = threadIdx.x;
    if (t < 4) bounds[kBoundsStat + t] = 0u;       // (the cut plan's stats: none unless one is made below)
    if (t == 0) {
        // (read and re-armed for the next joint count; the other threads read s_rows after a barrier)
        s_rows = (rows_cnt != nullptr && ctab != nullptr && rowone != nullptr && *rows_cnt == R) ? 1u : 0u;
        if (rows_cnt != nullptr) *rows_cnt = 0u;
    }
    if (enable != nullptr && *enable == kGroupsFixed) {  // no joint count this pass
        if (t == 0) bounds[0] = kGroupsFixed;
        return;
    }
    const uint32_t g = t % R, q = t / R;
    uint32_t s = 0, mx = 0;
    float sq = 0.f;
    for (uint32_t e = q * (R / Q); e < (q + 1) * (R / Q); ++e) {
        const uint32_t v = joint[e * R + g];
        s += v;
        mx = max(mx, v);
        sq += (float)v * (float)v;
    }
    s_part[q][g] = s;
    s_sq[q][g] = sq;
    s_mx[q][g] = mx;
    if (t == 0) s_max = 0u;
    __syncthreads();
    uint32_t tot = 0;
    if (t < R) {
#pragma unroll
        for (uint32_t i = 0; i < Q; ++i) tot += s_part[i][t];
        atomicMax(&s_max, tot);
    }
    uint32_t total = 0;
    const uint32_t start = block_excl_scan<1024>(tot, s_ws, total);
    if ((uint64_t)total != n) {
        if (t == 0) bounds[0] = kGroupsFixed;
        return;
    }
    if ((uint64_t)s_max <= max_keys) {
        if (t < R) bounds[1 + t] = start;
        if (t == 0) {
            bounds[1 + R] = total;
            bounds[0] = kGroupsWhole;
        }
        return;
    }
    // ---- cut plan: chunk c starts near c * n / R
    if (plan == nullptr) {  // (callers without a plan area: fixed chunks)
        if (t == 0) bounds[0] = kGroupsFixed;
        return;
    }
    if (t < R) {
        s_b[t] = start;
        s_big[t] = 0ull;
        s_cf[t] = 0xFFFFFFFFu;
        s_cl[t] = 0u;
    }
    if (t == 0) s_b[R] = total;
    __syncthreads();
    // the group holding position x < n: the last g with s_b[g] <= x (its end is past x)
    auto group_of = [&](uint32_t x) {
        uint32_t lo = 0, hi = R - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (s_b[mid] <= x) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    // weighted plans: per group the cost per key from its next-digit distribution, and the groups'
    // first weighted keys (units of 4 weighted keys: the total stays below 2^32)
    uint32_t WK = 0;
    if (weighted) {
        uint32_t wk = 0;
        if (t < R) {
            float w = 1.f;
            if (tot > 0) {
                float sqs = 0.f;
                uint32_t m = 0;
#pragma unroll
                for (uint32_t i = 0; i < Q; ++i) {
                    sqs += s_sq[i][t];
                    m = max(m, s_mx[i][t]);
                }
                const float inv = 1.f / (float)tot, top = (float)m * inv, h = sqs * inv * inv;
                w = (427.1f + 685.9f * fmaxf(h - top * top, 0.f) + 17.6f * top - 37.2f * top * top) / 427.1f;
                w = fminf(fmaxf(w, 0.8f), 1.4f);
            }
            s_w[t] = w;
            wk = (uint32_t)((float)tot * w * 0.25f);
        }
        const uint32_t c0 = block_excl_scan<1024>(wk, s_ws, WK);
        if (t < R) s_C[t] = c0;
        if (t == 0) s_C[R] = WK;
        __syncthreads();
    }
    if (t <= R) {
        uint32_t B = (uint32_t)((n * t) / R);
        if (weighted && t > 0 && t < R) {
            // the position where the weighted keys reach t / R of their total: the last group starting
            // at or below that weight, and inside it by its cost per key
            const uint32_t target = (uint32_t)(((uint64_t)WK * t) / R);
            uint32_t lo = 0, hi = R - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (s_C[mid] <= target) lo = mid;
                else hi = mid - 1;
            }
            const float off = (float)(target - s_C[lo]) * 4.f / s_w[lo];
            const uint32_t len = s_b[lo + 1] - s_b[lo];
            B = s_b[lo] + min((uint32_t)off, len);
        }
        if (t > 0 && t < R) {
            // snap to the nearer group boundary when it is within `snap` keys
            const uint32_t gg = group_of(B);
            const uint32_t d0 = B - s_b[gg], d1 = s_b[gg + 1] - B;
            if (min(d0, d1) <= snap) B = d0 <= d1 ? s_b[gg] : s_b[gg + 1];
        }
        s_B[t] = B;
        bounds[1 + t] = B;
    }
    __syncthreads();
    // per chunk: its first and last group and their segments in it
    uint32_t gA = 0, gB = 0, hb = 0, he = 0, tb = 0, te = 0;
    bool empty = true, hpart = false, tpart = false;
    if (t < R) {
        const uint32_t b = s_B[t], e = s_B[t + 1];
        empty = b >= e;
        if (!empty) {
            gA = group_of(b);
            gB = group_of(e - 1);
            hb = b;
            he = min(e, s_b[gA + 1]);
            hpart = hb > s_b[gA] || he < s_b[gA + 1];
            if (gB != gA) {
                tb = s_b[gB];
                te = e;
                tpart = te < s_b[gB + 1];
            }
            if (hpart) {
                atomicMax(&s_big[gA], ((unsigned long long)(he - hb) << 10) | (2u * t));
                atomicMin(&s_cf[gA], t);
                atomicMax(&s_cl[gA], t);
            }
            if (tpart) {
                atomicMax(&s_big[gB], ((unsigned long long)(te - tb) << 10) | (2u * t + 1u));
                atomicMin(&s_cf[gB], t);
                atomicMax(&s_cl[gB], t);
            }
        }
    }
    __syncthreads();
    // each cut group's largest segment is derived, the others are counted
    uint32_t hm = kSegWhole, tm = kSegWhole;
    if (hpart) hm = (uint32_t)(s_big[gA] & 1023u) == 2u * t ? kSegDerived : kSegCounted;
    if (tpart) tm = (uint32_t)(s_big[gB] & 1023u) == 2u * t + 1u ? kSegDerived : kSegCounted;
    // a counted piece [ps, pe) of group g: with rows, the previous pass's chunks wholly inside it are a
    // row task (chunk c's keys of group g sit at ctab[g][c] .. ctab[g][c + 1], the scanned table) and
    // only its two ends are key ranges -- each end, or the rest of the chunk it lies in when that is
    // shorter (the chunk's row then joins the task and the rest is counted negatively: a hot key's run
    // can fill a whole chunk's part of its group); else one key range
    struct Split {
        uint32_t b[2], e[2], neg[2];  // key ranges [b, e), counted negatively where neg
        uint32_t c0, c1;              // rows of chunks [c0, c1)
        uint32_t dl[2], de[2];        // direct adds: dl keys of next digit de (an end in a one-digit row)
    };
    const bool rows = s_rows != 0u;
    auto split = [&](uint32_t g, uint32_t ps, uint32_t pe) {
        Split sp{{ps, pe}, {pe, pe}, {0u, 0u}, 0u, 0u, {0u, 0u}, {0u, 0u}};
        if (!rows) return sp;
        const uint32_t *row = ctab + (uint64_t)g * R;
        const uint32_t gend = s_b[g + 1];
        auto P = [&](uint32_t cc) { return cc < R ? row[cc] : gend; };
        uint32_t lo = 0, hi = R;  // first boundary >= ps
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (P(mid) >= ps) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t c0 = lo;
        lo = 0;
        hi = R;  // last boundary <= pe
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (P(mid) <= pe) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t c1 = lo;
        auto one = [&](uint32_t cc) { return rowone[(uint64_t)cc * R + g]; };  // chunk cc's row: its one digit
        if (c0 <= c1) {
            // whole chunks [c0, c1); the left end [ps, P(c0)) lies in chunk c0 - 1, the right end
            // [P(c1), pe) in chunk c1 (P(0) <= ps and pe <= P(R): the chunks exist when the ends do)
            sp = Split{{ps, P(c1)}, {P(c0), pe}, {0u, 0u}, c0, c1, {0u, 0u}, {0u, 0u}};
            if (ps < P(c0)) {
                const uint32_t e1 = one(c0 - 1);
                if (e1 < R) {
                    sp.dl[0] = P(c0) - ps;
                    sp.de[0] = e1;
                    sp.b[0] = sp.e[0];
                } else if (ps - P(c0 - 1) < P(c0) - ps) {
                    sp.b[0] = P(c0 - 1);
                    sp.e[0] = ps;
                    sp.neg[0] = 1u;
                    sp.c0 = c0 - 1;
                }
            }
            if (pe > P(c1)) {
                const uint32_t e2 = one(c1);
                if (e2 < R) {
                    sp.dl[1] = pe - P(c1);
                    sp.de[1] = e2;
                    sp.b[1] = sp.e[1];
                } else if (P(c1 + 1) - pe < pe - P(c1)) {
                    sp.b[1] = pe;
                    sp.e[1] = P(c1 + 1);
                    sp.neg[1] = 1u;
                    sp.c1 = c1 + 1;
                }
            }
        } else if (one(c1) < R) {
            // inside chunk c1 = c0 - 1, whose keys of group g all have one next digit
            sp = Split{{pe, pe}, {pe, pe}, {0u, 0u}, 0u, 0u, {pe - ps, 0u}, {one(c1), 0u}};
        } else if (P(c0) - P(c1) < 2 * (pe - ps)) {
            // inside chunk c1, and its rest is the shorter: its row less the two rest ranges
            sp = Split{{P(c1), pe}, {ps, P(c0)}, {1u, 1u}, c1, c0, {0u, 0u}, {0u, 0u}};
        }
        return sp;
    };
    Split hs{{0u, 0u}, {0u, 0u}, {0u, 0u}, 0u, 0u, {0u, 0u}, {0u, 0u}}, ts = hs;
    if (hm == kSegCounted) hs = split(gA, hb, he);
    if (tm == kSegCounted) ts = split(gB, tb, te);
    const uint32_t npc = (hm == kSegCounted ? 1u : 0u) + (tm == kSegCounted ? 1u : 0u);
    auto nranges = [](const Split &x) { return (x.e[0] > x.b[0] ? 1u : 0u) + (x.e[1] > x.b[1] ? 1u : 0u); };
    auto nkeys = [](const Split &x) {
        return (x.e[0] > x.b[0] ? x.e[0] - x.b[0] : 0u) + (x.e[1] > x.b[1] ? x.e[1] - x.b[1] : 0u);
    };
    const uint32_t nrg = nranges(hs) + nranges(ts);
    const uint32_t nkc = nkeys(hs) + nkeys(ts);
    auto ntasks = [](const Split &x) {
        return (x.c1 > x.c0 ? 1u : 0u) + (x.dl[0] > 0u ? 1u : 0u) + (x.dl[1] > 0u ? 1u : 0u);
    };
    const uint32_t nrt = ntasks(hs) + ntasks(ts);
    uint32_t np = 0, K = 0, nr = 0, npieces = 0;
    uint32_t pi = block_excl_scan<1024>(npc, s_ws, npieces);
    uint32_t gi = block_excl_scan<1024>(nrg, s_ws, np);
    uint32_t ko = block_excl_scan<1024>(nkc, s_ws, K);
    uint32_t ri = block_excl_scan<1024>(nrt, s_ws, nr);
    if (t < R) {
        plan[kPlanDesc + t] = gA | (gB << 8) | (hm << 16) | (tm << 18) | ((empty ? 1u : 0u) << 20);
        plan[kPlanGroup + t] = (s_cf[t] & 255u) | ((s_cl[t] & 255u) << 8) | ((uint32_t)(s_big[t] & 1023u) << 16);
        auto emit = [&](const Split &x, uint32_t sl, uint32_t g) {
            for (int i = 0; i < 2; ++i) {
                if (x.e[i] <= x.b[i]) continue;
                uint32_t *pc = plan + kPlanPieces + 4 * gi;
                pc[0] = x.b[i];
                pc[1] = x.e[i];
                pc[2] = sl | (x.neg[i] ? kPieceNeg : 0u);
                pc[3] = ko;
                ++gi;
                ko += x.e[i] - x.b[i];
            }
            if (x.c1 > x.c0) {
                uint32_t *rt = plan + kPlanRows + 4 * ri;
                rt[0] = sl;
                rt[1] = g;
                rt[2] = x.c0;
                rt[3] = x.c1;
                ++ri;
            }
            for (int i = 0; i < 2; ++i) {
                if (x.dl[i] == 0u) continue;
                uint32_t *rt = plan + kPlanRows + 4 * ri;  // a direct add: dl keys of next digit de
                rt[0] = sl;
                rt[1] = kRowDirect | x.de[i];
                rt[2] = x.dl[i];
                rt[3] = 0u;
                ++ri;
            }
        };
        if (hm == kSegCounted) {
            emit(hs, (2u * t) | ((uint32_t)(s_big[gA] & 1023u) << 16), gA);
            s_slot[pi] = 2u * t;
            ++pi;
        }
        if (tm == kSegCounted) {
            emit(ts, (2u * t + 1u) | ((uint32_t)(s_big[gB] & 1023u) << 16), gB);
            s_slot[pi] = 2u * t + 1u;
        }
    }
    np = min(np, kPlanMaxRanges);  // (cannot exceed it: <= 255 counted pieces, 2 ranges each)
    // the plan's make-up for rsort_cut_plan_stats (tests): direct adds and negatively counted ranges
    auto ndirect = [](const Split &x) { return (x.dl[0] > 0u ? 1u : 0u) + (x.dl[1] > 0u ? 1u : 0u); };
    auto nneg = [](const Split &x) {
        return (x.neg[0] && x.e[0] > x.b[0] ? 1u : 0u) + (x.neg[1] && x.e[1] > x.b[1] ? 1u : 0u);
    };
    uint32_t ndir = 0, nng = 0;
    (void)block_excl_scan<1024>(t < R ? ndirect(hs) + ndirect(ts) : 0u, s_ws, ndir);
    (void)block_excl_scan<1024>(t < R ? nneg(hs) + nneg(ts) : 0u, s_ws, nng);
    if (t == 0) {
        plan[0] = np;
        plan[1] = K;
        plan[2] = nr;
        bounds[0] = kGroupsCut;
        bounds[kBoundsStat] = np;
        bounds[kBoundsStat + 1] = nr - ndir;
        bounds[kBoundsStat + 2] = ndir;
        bounds[kBoundsStat + 3] = nng;
    }
    __syncthreads();
    // the counted pieces' rows and each cut group's derived row start at zero (the histogram
    // launch adds every piece's counts into its row and takes them from its group's derived row)
    for (uint32_t i = t; i < npieces * R; i += 1024) pcounts[s_slot[i / R] * R + i % R] = 0u;
    for (uint32_t i = t; i < R * R; i += 1024) {
        const uint32_t gg = i / R, d = i % R;
        if (s_big[gg] != 0ull) pcounts[(uint32_t)(s_big[gg] & 1023u) * R + d] = 0u;
    }
}

// ------------------------------------------------------------------------------ scatter
// Reference: sortLocallyDataBlocks (P7:193-251: scanLocallyBlocksUnroll2Kernel :79-141 +
// scatterLocallyBlocksKernel :143-191, or the in-SMEM P5:79-159) fused with scatterKernel
// (P7:253-304). Per tile: load (coalesced, wave-striped: lane l of wave w holds tile
// positions w*64*KPT + j*64 + l), rank locally, stage the tile in LDS in digit order, then
// write each digit's run to global at table[digit][chunk] + (earlier tiles' count) +
// (position - first position of the digit in the tile) -- the firstIndices rank formula of
// P7:293-294 with the running offset kept in registers.
//
// This is the general pass (any k, unaligned outputs, local-only mode, the reference's 1-bit
// split ranking); the k = 3..8 sorts with 16-B aligned buffers run rs_scatter_lines below.
//   RANK  kRankAtomic  count first (per-wave LDS digit counters), scan them into tile positions,
//                      then one returning LDS add per key: the lane-ordered add IS the key's
//                      stable position (rank_add)
//         kRankCount   the same with the wave64 ballot peer match instead of the lane order
//         kRankSplit   k stable 1-bit splits (the reference's algorithm)
//   MINW  minimum waves per SIMD requested from the register allocator (0 = compiler's choice)
template <int BITS, int THREADS, int KPT, bool PAIRS, int RANK, int DMODE, int MINW = 0>
__global__ __launch_bounds__(THREADS, MINW > 0 ? MINW : 1) void rs_scatter(ScatterArgs a) {
    constexpr bool COUNT_FIRST = (RANK == kRankCount || RANK == kRankAtomic);
    static_assert(COUNT_FIRST || RANK == kRankSplit, "ranking variant");
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int SEG = kWave * KPT;            // tile positions per wave
    constexpr uint32_t T = THREADS * KPT;       // tile keys
    constexpr int DPT = (R > THREADS) ? (int)(R / THREADS) : 1;  // digits owned per thread
    constexpr uint32_t NCNT = COUNT_FIRST ? W * R : R;

    __shared__ uint32_t s_keys[T];
    __shared__ uint32_t s_vals[PAIRS ? T : 1];
    __shared__ uint16_t s_aux[RANK == kRankSplit ? T : 1];
    __shared__ uint32_t s_cnt[NCNT];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_ws[W];

    const uint32_t t = threadIdx.x;
    const uint32_t w = t / kWave;
    const uint32_t lane = lane_id();
    const uint32_t c = blockIdx.x;
    const Digit<BITS, DMODE> dig{a.shift, a.nsplit, a.splitters};
    const uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    const uint64_t cend = min(cbeg + a.chunk_keys, a.n);

    // Running global offset of each owned digit (thread t owns digits t*DPT .. t*DPT+DPT-1,
    // or digit t when R < THREADS).
    uint32_t run[DPT];
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
        const uint32_t d = t * DPT + i;
        run[i] = (d < R && !a.local_only) ? a.table[(uint64_t)d * a.num_chunks + c] : 0u;
    }

    const uint32_t base = w * SEG + lane;
    // Tile loader: positions past the end read as 0xFFFFFFFF, whose digit is the largest
    // possible one, so they rank after every real key of the tile and are never written out.
    auto load_tile = [&](uint64_t tb, uint32_t (&k)[KPT], uint32_t (&v)[PAIRS ? KPT : 1]) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        // wave-uniform tile base + 32-bit lane offsets: saddr loads with immediate offsets, no
        // per-slot 64-bit address registers kept alive across the tile loop
        const uint32_t *__restrict__ tk = a.kin + tb;
        const uint32_t *__restrict__ tv = PAIRS ? a.vin + tb : nullptr;
        if (valid == T) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                k[j] = tk[base + j * kWave];
                if constexpr (PAIRS) v[j] = tv[base + j * kWave];
            }
        } else {
            // lane-relative limit: slot j is real iff j*64 < lim (no per-slot offset registers)
            const uint32_t lim = valid > base ? valid - base : 0u;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool in = (uint32_t)(j * kWave) < lim;
                k[j] = in ? tk[base + j * kWave] : 0xFFFFFFFFu;
                if constexpr (PAIRS) v[j] = in ? tv[base + j * kWave] : 0u;
            }
        }
    };

    uint32_t key[KPT];
    uint32_t val[PAIRS ? KPT : 1];
    if (cbeg < cend) load_tile(cbeg, key, val);
    uint32_t order_bad = 0;  // kRankAtomic: the per-tile rank check (rank_check) failed in this thread

    for (uint64_t tb = cbeg, tno = 0; tb < cend; tb += T, ++tno) {
        // the rank check on every kRankCheckEvery-th tile of a chunk, its first included (workgroup-uniform)
        const bool check_tile = (tno & (kRankCheckEvery - 1)) == 0;
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        // tl: the thread index made opaque per tile, so LICM cannot hoist the KPT output
        // positions tl + j*THREADS out of the loop into KPT live registers; output slot j of
        // thread t (LDS position t + j*THREADS) is real iff j*THREADS < olim
        uint32_t tl = t;
        asm volatile("" : "+v"(tl));
        const uint32_t olim = valid > tl ? valid - tl : 0u;
        const uint64_t nb = tb + T;

        if constexpr (!COUNT_FIRST) {
            for (uint32_t i = t; i < NCNT; i += THREADS) s_cnt[i] = 0;
            __syncthreads();
        }

        if constexpr (COUNT_FIRST) {
            // ---- 0. each wave clears its own counters: no other wave touches s_cnt[w][*]
            //      between the previous tile's digit scan (behind two barriers) and this point
#pragma unroll
            for (uint32_t i = lane; i < R; i += kWave) s_cnt[w * R + i] = 0;
            // ---- 1. per-wave digit histogram of the tile
#pragma unroll
            for (int j = 0; j < KPT; ++j) count_add(&s_cnt[w * R], dig(key[j]));
            __syncthreads();
            // ---- 2. digit scan: s_cnt[w][d] <- tile position of wave w's first key of digit d
            uint32_t tot[DPT];
            uint32_t mine = 0;
#pragma unroll
            for (int i = 0; i < DPT; ++i) {
                const uint32_t d = t * DPT + i;
                uint32_t acc = 0;
                if (d < R) {
#pragma unroll
                    for (int v = 0; v < W; ++v) {
                        const uint32_t x = s_cnt[v * R + d];
                        s_cnt[v * R + d] = acc;
                        acc += x;
                    }
                }
                tot[i] = acc;
                mine += acc;
            }
            uint32_t all;
            uint32_t start = block_excl_scan<THREADS>(mine, s_ws, all);
#pragma unroll
            for (int i = 0; i < DPT; ++i) {
                const uint32_t d = t * DPT + i;
                if (d < R) {
#pragma unroll
                    for (int v = 0; v < W; ++v) s_cnt[v * R + d] += start;
                    s_delta[d] = run[i] - start;
                    run[i] += tot[i];
                }
                start += tot[i];
            }
            __syncthreads();
            // ---- 3. rank each slot; the counter IS the destination: write the key now
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                // recompute the digit: CSE with the histogram step would keep KPT addresses alive
                asm volatile("" : "+v"(key[j]));
                const uint32_t d = dig(key[j]);
                if constexpr (RANK == kRankAtomic) {
                    // one returning LDS add per key: gfx950 serves the lanes of a ds_add_rtn_u32
                    // that hit the same address in ascending lane order, so lane l receives
                    // base + (#lower lanes with its digit) -- the stable rank, with no ballots
                    // (rank_add; the library probes this once per device, rs_lane_order_probe)
                    uint32_t p = rank_add(&s_cnt[w * R], d);
                    if (j == 0 && valid == T && check_tile) order_bad |= rank_check<BITS>(d, p, a.rank_fault);
                    s_keys[p] = key[j];
                    if constexpr (PAIRS) s_vals[p] = val[j];
                    continue;
                }
                uint32_t mlo, mhi;
                peer_mask<BITS>(d, mlo, mhi);
                const uint32_t pre = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
                const uint32_t old = s_cnt[w * R + d];
                if (pre == 0) s_cnt[w * R + d] = old + (uint32_t)(__builtin_popcount(mlo) + __builtin_popcount(mhi));
                s_keys[old + pre] = key[j];
                if constexpr (PAIRS) s_vals[old + pre] = val[j];
            }
            __syncthreads();
            if (nb < cend) load_tile(nb, key, val);
            if (a.local_only) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t i = tl + j * THREADS;
                    if ((uint32_t)(j * THREADS) < olim) {
                        a.kout[tb + i] = s_keys[i];
                        if constexpr (PAIRS) a.vout[tb + i] = s_vals[i];
                    }
                }
            } else {
                const bool full = valid == T;
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t i = tl + j * THREADS;
                    if (full || (uint32_t)(j * THREADS) < olim) {
                        const uint32_t k = s_keys[i];
                        const uint32_t pos = s_delta[dig(k)] + i;
                        a.kout[pos] = k;
                        if constexpr (PAIRS) a.vout[pos] = s_vals[i];
                    }
                    // issue the output in groups of 8 keys: bounds the LDS reads in flight
                    if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else {
            // ---- RANK_SPLIT: k stable 1-bit splits in LDS (reference P5:89-146 / P7:79-191)
            uint32_t dg[KPT];
#pragma unroll
            for (int j = 0; j < KPT; ++j) dg[j] = dig(key[j]);  // padding 0xFFFFFFFF -> the largest digit
            const uint64_t below = lanes_below();
#pragma unroll 1
            for (int b = 0; b < BITS; ++b) {
                uint32_t wones = 0;
                uint32_t olt[KPT];
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint64_t bal = __ballot((dg[j] >> b) & 1u);
                    olt[j] = wones + (uint32_t)__popcll(bal & below);
                    wones += (uint32_t)__popcll(bal);
                }
                if (lane == 0) s_ws[w] = wones;
                __syncthreads();
                uint32_t pre = 0, ones = 0;
#pragma unroll
                for (int v = 0; v < W; ++v) {
                    const uint32_t s = s_ws[v];
                    pre += ((uint32_t)v < w) ? s : 0u;
                    ones += s;
                }
                const uint32_t zeros = T - ones;
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t p = base + j * kWave;
                    const uint32_t ob = pre + olt[j];  // ones before position p
                    const uint32_t np = ((dg[j] >> b) & 1u) ? zeros + ob : p - ob;
                    s_keys[np] = key[j];
                    s_aux[np] = (uint16_t)dg[j];
                    if constexpr (PAIRS) s_vals[np] = val[j];
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t p = base + j * kWave;
                    key[j] = s_keys[p];
                    dg[j] = s_aux[p];
                    if constexpr (PAIRS) val[j] = s_vals[p];
                }
            }
            // ---- tile digit counts -> first position of each digit (firstIndices, P7:267-288)
#pragma unroll
            for (int j = 0; j < KPT; ++j) atomicAdd(&s_cnt[dg[j]], 1u);
            __syncthreads();
            uint32_t tot[DPT];
            uint32_t mine = 0;
#pragma unroll
            for (int i = 0; i < DPT; ++i) {
                const uint32_t d = t * DPT + i;
                tot[i] = (d < R) ? s_cnt[d] : 0u;
                mine += tot[i];
            }
            uint32_t all;
            uint32_t start = block_excl_scan<THREADS>(mine, s_ws, all);
#pragma unroll
            for (int i = 0; i < DPT; ++i) {
                const uint32_t d = t * DPT + i;
                if (d < R) {
                    s_delta[d] = run[i] - start;
                    run[i] += tot[i];
                }
                start += tot[i];
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t p = base + j * kWave;
                if (p < valid) {
                    const uint64_t pos = a.local_only ? tb + p : (uint64_t)(s_delta[dg[j]] + p);
                    a.kout[pos] = key[j];
                    if constexpr (PAIRS) a.vout[pos] = val[j];
                }
            }
            if (nb < cend) load_tile(nb, key, val);
        }
    }
    if constexpr (RANK == kRankAtomic) report_order(a.check, order_bad);
}

// ------------------------------------------------------------------------------ raw-table offsets
// Next-digit plans (k = 3, 4), passes after the first: `table` holds the counts [d][c'] the previous
// pass ADDED (unscanned). Every workgroup derives its own starts s_base[d] = (keys of every digit
// below d) + (keys of digit d in chunks before c) from the whole table (R x C words: 64 KB at C2,
// held in each XCD's L2 after the first reads) instead of one workgroup scanning it at the end of the
// previous pass (tail_scan: ~5 us on the critical path of every pass). TPR = THREADS / R threads per
// row, each summing every TPR-th quad of it, 8 quads in flight; the caller issues its first tile's
// loads before (C2: 0.1183 vs 0.1206 ms per pass against one quad at a time behind no loads,
// dev/lab.sh ab). Returns false (in every thread) when the table does not
// hold exactly n keys: the caller then writes nothing (no offset can leave the output), and workgroup
// 0 records it for rsort_plan_check. All threads must call it; ends with a barrier.
template <int THREADS, uint32_t R>
__device__ bool raw_offsets(const uint32_t *table, uint32_t C, uint32_t c, uint64_t n, uint32_t *s_base,
                            uint32_t *s_tot, uint32_t *err) {
    constexpr uint32_t TPR = THREADS / R;
    static_assert(TPR >= 1 && TPR <= (uint32_t)kWave && (TPR & (TPR - 1)) == 0, "a row's threads in one wave");
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t t = threadIdx.x, d = t / TPR, sub = t % TPR;
    const uint32_t *row = table + (uint64_t)d * C;
    uint32_t all = 0, below = 0;
    if ((C & 3u) == 0u) {  // (rows start 16-B aligned: the table is)
        const u32x4 *r4 = reinterpret_cast<const u32x4 *>(row);
        const uint32_t nq = C / 4u;
        constexpr uint32_t RB = 8;  // quads in flight per thread
        for (uint32_t q0 = sub; q0 < nq; q0 += RB * TPR) {
            u32x4 v[RB];
#pragma unroll
            for (uint32_t i = 0; i < RB; ++i) {
                const uint32_t q = q0 + i * TPR;
                v[i] = q < nq ? r4[q] : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (uint32_t i = 0; i < RB; ++i) {
                const uint32_t c0 = (q0 + i * TPR) * 4u;
                all += v[i].x + v[i].y + v[i].z + v[i].w;
                below += (c0 < c ? v[i].x : 0u) + (c0 + 1u < c ? v[i].y : 0u) + (c0 + 2u < c ? v[i].z : 0u) +
                         (c0 + 3u < c ? v[i].w : 0u);
            }
        }
    } else {
        for (uint32_t x = sub; x < C; x += TPR) {
            const uint32_t v = row[x];
            all += v;
            below += x < c ? v : 0u;
        }
    }
    uint32_t p0, tall, tbelow;
    group_scan<TPR>(all, sub, p0, tall);
    group_scan<TPR>(below, sub, p0, tbelow);
    if (sub == 0) {
        s_tot[d] = tall;
        s_base[d] = tbelow;
    }
    __syncthreads();
    uint64_t tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < R; ++i) tot += s_tot[i];  // (every thread: the same sum)
    if (t < R) {
        uint32_t pre = 0;
#pragma unroll
        for (uint32_t i = 0; i < R; ++i) pre += i < t ? s_tot[i] : 0u;
        s_base[t] += pre;
        if (c == 0 && t == 0 && tot != n && err != nullptr) atomicOr(err, kCheckTable);
    }
    __syncthreads();
    return tot == n;
}

// ------------------------------------------------------------------------------ small kernels
// starts[d] = scanned table[d][0] (global start of digit d), starts[bins] = n.
// ------------------------------------------------------------------------------ scatter (line-combining)
// rs_scatter_lines: the same pass as rs_scatter (Parallel7.cu:193-316 fused), built so that every
// global store is a whole, aligned G-key line written by 16-B-per-lane store instructions.
// A digit's output region inside a chunk is contiguous, but each tile ends it mid-line; writing
// those partial lines costs as much HBM time as whole ones (dev/wc_lab.hip: 1.7 ms aligned vs
// 2.8 ms misaligned for the same 8 GB). So each digit carries the < G keys past its last whole
// line into the next tile.
//
// Per tile (count-first ranking, one returning LDS atomic per key -- see kRankAtomic):
//   1. per-wave digit histogram (non-returning LDS adds)
//   2. per digit: pending output = carry (c keys from the line-aligned A = g - c) + this tile's
//      run; its whole lines occupy an LDS segment [S, S + wcnt) whose start is line-aligned, so
//      LDS line L <-> one global line. The old carry is copied into the segment head, each line
//      gets a record {global key index, first valid lane}, the per-wave counters start after
//      the carry
//   3. rank + stage: P = atomicAdd(counter) is the key's LDS slot; slots past the last whole
//      line (P >= lim) go to the digit's carry (one store, the address selected)
//   4. output: 4 keys per lane, ds_read_b128 + global_store_dwordx4, G/4 lanes per line
// At a chunk's start the carry is the (invalid) part of the first line that precedes the
// chunk's output, so that line is written with a lane mask; after the chunk's last tile the
// remaining carries are flushed with masked dword stores (both lines are shared with the
// neighbouring chunks' output). Only the grid's very last tile is partial (chunks are whole
// tiles), so the full-tile paths carry no per-slot predicates.
template <int BITS, int THREADS, int KPT, int G, bool PAIRS, int DMODE, int NT = 0, int CL = 0>
__global__ __launch_bounds__(THREADS, THREADS == 256 ? hooks::kLinesMinWavesSmall : 1) void rs_scatter_lines(ScatterArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int SEG = kWave * KPT;
    constexpr uint32_t T = THREADS * KPT;
    constexpr uint32_t TPD = THREADS / R;            // threads per digit
    constexpr uint32_t CAP = T + (G - 1) * R;        // staged keys incl. carries, worst case
    constexpr uint32_t NL = CAP / G;
    constexpr uint32_t QPL = G / 4;                  // 16-B quads per line
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    static_assert(R <= THREADS && TPD <= kWave && (G == 16 || G == 32),
                  "a digit's thread group lies in one wave; 64/128-B lines");
    static_assert(CAP + R * G < 65536u, "LDS slot indices are packed in 16 bits");

    // staging: [0, CAP) whole lines of every digit, [CAP, CAP + R*G) the per-digit carries
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[CAP + R * G + 4];  // + padding sink
    __shared__ __attribute__((aligned(16))) uint32_t s_vstage[PAIRS ? CAP + R * G + 4 : 4];
    // per-wave counter rows RS >= R words apart (counter_stride): step 2's digit-group threads read
    // and write rows sub * WPT + i of their digit's column, which R apart share one bank
    constexpr uint32_t RS = counter_stride<R, TPD, (W >= (int)TPD) ? W / TPD : 0>();
    __shared__ uint32_t s_cnt[W * RS + 1];                                       // + padding counter
    // per digit: {global - LDS key index, first line << 8 | first valid lane} (+ with next-digit counts, s_nb's
    // position: one LDS read per output quad gets both)
    typedef typename std::conditional<(R <= 16) && DMODE == kDigitShift, uint4, uint2>::type OutRec;
    __shared__ OutRec s_out[R];
    __shared__ uint2 s_flush[R];      // chunk end: {A, inv | carry << 8}
    __shared__ uint32_t s_ws[W];
    // Next-digit counts (k <= 4 with a.next_table): the NEXT pass's chunk table, counted here by
    // where each key is written. Digit d's keys of this chunk land in [table[d][c], + count) --
    // at most chunk_keys keys, so in at most two of the next pass's chunks (same plan, same
    // chunks): s_next[(d * 2 + slot) * R + next digit], slot 1 from position s_nb[d] on. The
    // next pass then reads no keys for its histogram.
    // NXR replicas of every counter, picked by lane % NXR: the lanes of one output instruction mostly
    // share (digit, slot) -- a digit's lines are adjacent -- so without them ~4 lanes would hit
    // each of the R counters and serialise in the LDS
    constexpr bool NX = (R <= 16) && DMODE == kDigitShift;
    constexpr uint32_t NXR = hooks::kNextReplicas;
    __shared__ uint32_t s_next[NX ? 2 * R * R * NXR : 1];
    __shared__ uint32_t s_nb[NX ? R : 1];  // first position of digit d's second output chunk
    __shared__ uint32_t s_oc[NX ? R : 1];  // digit d's first output chunk
    const bool count_next = NX && a.next_table != nullptr;
    __shared__ uint32_t s_base[NX ? R : 1];  // raw-table offsets (ScatterArgs::raw_table)
    __shared__ uint32_t s_rtot[NX ? R : 1];

    const uint32_t t = threadIdx.x;
    const uint32_t w = t / kWave;
    const uint32_t lane = lane_id();
    const uint32_t c = blockIdx.x;
    // 16-bucket split digits from the prefix table (Digit::fill_table; built before the first tile's
    // ranking). With <= 7 splitters the compares are cheaper than the table's LDS read (2^30 keys into 8
    // buckets: 1.79 ms with compares, 1.83 with the table; into 16: 2.25 with compares, 1.74 with it)
    constexpr bool STAB = DMODE == kDigitSplit && BITS > 3;
    __shared__ uint32_t s_stab[STAB ? kSplitTabWords : 1];
    const Digit<BITS, DMODE> dig{a.shift, a.nsplit, a.splitters, STAB ? s_stab : nullptr};
    uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    uint32_t head = 0;  // leading keys of the first tile that belong to the previous chunk
    // clustered-pass selection (ScatterArgs::cl_select): the plain and the clustered kernel are both
    // launched, and the one not selected by the device-side flag leaves at once
    if (a.cl_select != nullptr && ((*a.cl_select != kGroupsWhole) != (CL != 0))) return;
    RS_WG_T0
    if (a.bounds != nullptr && a.bounds[0] != 0u) {
        // digit-group chunk (rs_histogram_joint): any start, so the tiles start at the 256-B
        // boundary below it (every wave load stays two whole 128-B lines), the first tile skips
        // its `head` keys, and every chunk may end in a partial tile
        const uint64_t b = a.bounds[1 + c];
        cend = a.bounds[2 + c];
        cbeg = b < cend ? (b & ~(uint64_t)(kWave - 1)) : cend;
        head = (uint32_t)(b < cend ? b - cbeg : 0);
    }

    // digit group of this thread: digit d = t / TPD; the leader (sub == 0) keeps the state
    const uint32_t d_own = t / TPD;
    const uint32_t sub = t % TPD;
    const bool leader = sub == 0;
    const uint32_t glead = lane & ~(TPD - 1u);
    uint32_t g_run = 0, carry = 0, inv = 0, nb_own = 0;  // (nb_own: the leader's s_nb entry)
    const uint32_t base = w * SEG + lane;
    auto load_tile = [&](uint64_t tb, uint32_t (&k)[KPT], uint32_t (&v)[PAIRS ? KPT : 1]) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        uint32_t lb = base;  // opaque: one lane offset + immediate slot offsets, nothing hoisted
        asm volatile("" : "+v"(lb));
        const uint32_t *__restrict__ tk = a.kin + tb + lb;
        const uint32_t *__restrict__ tv = PAIRS ? a.vin + tb + lb : nullptr;
        if (valid == T) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                // NT & 1: non-temporal key/value loads (dev/scatter_lab experiment)
                k[j] = (NT & 1) ? __builtin_nontemporal_load(tk + j * kWave) : tk[j * kWave];
                if constexpr (PAIRS) v[j] = (NT & 1) ? __builtin_nontemporal_load(tv + j * kWave) : tv[j * kWave];
            }
        } else {
            const uint32_t lim = valid > lb ? valid - lb : 0u;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool in = (uint32_t)(j * kWave) < lim;
                k[j] = in ? tk[j * kWave] : 0u;
                if constexpr (PAIRS) v[j] = in ? tv[j * kWave] : 0u;
            }
        }
    };
    uint32_t key[KPT];
    uint32_t val[PAIRS ? KPT : 1];
    if (cbeg < cend) load_tile(cbeg, key, val);
    if constexpr (STAB) {
        dig.fill_table(t, THREADS);  // (while the first tile's loads are in flight)
        __syncthreads();
    }
    if constexpr (NX) {
        // this workgroup's share of the table the pass after next counts into (nobody reads that
        // one in this pass) is cleared on the way
        if (a.zero_table != nullptr)
            for (uint32_t i = t; i < R; i += THREADS) a.zero_table[(uint64_t)c * R + i] = 0u;
        // this workgroup's starts from the previous pass's raw counts (a table that does not hold n
        // keys -- never observed -- writes nothing: recorded for rsort_plan_check)
        if (a.raw_table &&
            !raw_offsets<THREADS, R>(a.table, a.num_chunks, c, a.n, s_base, s_rtot, a.done ? a.done + kDoneErr : nullptr))
            return;
    }
    if (leader) {
        // positions relative to kout's 128-B-aligned base (ScatterArgs::pos_shift): lines are cache lines
        uint32_t g0;
        if constexpr (NX) g0 = a.raw_table ? s_base[d_own] : a.table[(uint64_t)d_own * a.num_chunks + c];
        else g0 = a.table[(uint64_t)d_own * a.num_chunks + c];
        const uint32_t g = g0 + a.pos_shift;
        carry = g & (G - 1u);  // the first line starts before the chunk's output
        inv = carry;
        g_run = g;
        // the invalid slots get a key of this digit (never stored: masked), so every staged
        // slot's key tells the output phase its digit (a bucket's lower splitter in split mode;
        // a bucket whose splitter repeats is empty and writes no line)
        uint32_t ik = d_own << a.shift;
        if constexpr (DMODE == kDigitSplit)
            ik = (d_own == 0 || a.nsplit == 0) ? 0u : a.splitters[min(d_own, a.nsplit) - 1u];
        for (uint32_t x = 0; x < inv; ++x) s_stage[CAP + d_own * G + x] = ik;
        if constexpr (NX) {
            if (count_next) {
                const uint64_t oc = (uint64_t)g0 / a.chunk_keys;  // (the next pass's chunks: unshifted)
                s_oc[d_own] = (uint32_t)oc;
                nb_own = (uint32_t)min<uint64_t>((oc + 1) * a.chunk_keys, 0xFFFFFFFFull);
                s_nb[d_own] = nb_own;
            }
        }
    }
    if constexpr (NX) {
        if (count_next)
            for (uint32_t i = t; i < 2 * R * R * NXR; i += THREADS) s_next[i] = 0;
    }
    // one written key of digit d at global position gp: count its next digit (k <= 4 plans)
    auto next_add = [&](uint32_t d, uint32_t slot, uint32_t key) {
        const uint32_t e = (key >> (a.shift + BITS)) & (R - 1u);
        atomicAdd(&s_next[((d * 2 + slot) * R + e) * NXR + (lane & (NXR - 1))], 1u);
    };


    // one 16-B quad of line L at quad offset q -> global; every key of an LDS line has the line's
    // digit, which locates the line's segment record (info)
    auto store_quad = [&](uint32_t L, uint32_t q, const u32x4 &kv, const u32x4 &vv, const OutRec &info, uint32_t d) {
        const uint32_t lo = (info.y >> 8) == L ? (info.y & 0xFFu) : 0u;
        const uint64_t gp = (uint64_t)(info.x + L * G + q);
        if constexpr (NX) {
            if (count_next) {
                // (per element: with a pos_shift that is not a multiple of 4 a quad can straddle a
                // chunk boundary of the unshifted positions). s_nb[d] comes with the digit's record: read
                // inside the element loop it was re-read after every add (the adds may alias it), each
                // read a full LDS round trip the adds then waited for (k = 4 middle passes, dev/LOG.md)
                const uint32_t p0 = (uint32_t)gp - a.pos_shift;
                uint32_t nbd;
                if constexpr (NX) nbd = info.z;
                if (lo <= q) {  // (every element: all but a chunk's first line)
#pragma unroll
                    for (uint32_t x = 0; x < 4; ++x) next_add(d, p0 + x >= nbd ? 1u : 0u, kv[x]);
                } else {
#pragma unroll
                    for (uint32_t x = 0; x < 4; ++x)
                        if (lo <= q + x) next_add(d, p0 + x >= nbd ? 1u : 0u, kv[x]);
                }
            }
        }
        if (lo <= q) {
            if constexpr ((NT & 2) != 0) {  // non-temporal whole-line stores
                hooks::store_quad_nt(a.kout + gp, kv);
                if constexpr (PAIRS) hooks::store_quad_nt(a.vout + gp, vv);
            } else {
                hooks::store_quad(a.kout + gp, kv);
                if constexpr (PAIRS) hooks::store_quad(a.vout + gp, vv);
            }
        } else {
            // the chunk's first line: lanes below lo belong to the previous chunk
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x)
                if (lo <= q + x) {
                    hooks::store_word(a.kout + gp + x, kv[x]);
                    if constexpr (PAIRS) hooks::store_word(a.vout + gp + x, vv[x]);
                }
        }
    };
    // step 4's unit of work: two quads per thread and round (items t and t + THREADS): both LDS
    // reads, then both segment records, then both stores -- two independent chains in flight
    // instead of read -> wait -> record -> wait -> store per quad (dev/lines_exp.hip OUTB2: -1 % per
    // C3 pass; all of a thread's quads at once made the compiler wait for the stores: +60 %)
    auto out_pair = [&](uint32_t item, uint32_t nq) {
        const uint32_t i2 = item + THREADS;
        const bool two = i2 < nq;
        const uint32_t L0 = item / QPL, q0 = (item % QPL) * 4u, L1 = i2 / QPL, q1 = (i2 % QPL) * 4u;
        const u32x4 kv0 = *reinterpret_cast<const u32x4 *>(&s_stage[L0 * G + q0]);
        u32x4 kv1 = kv0, vv0 = kv0, vv1 = kv0;
        if (two) kv1 = *reinterpret_cast<const u32x4 *>(&s_stage[L1 * G + q1]);
        if constexpr (PAIRS) {
            vv0 = *reinterpret_cast<const u32x4 *>(&s_vstage[L0 * G + q0]);
            if (two) vv1 = *reinterpret_cast<const u32x4 *>(&s_vstage[L1 * G + q1]);
        }
        const uint32_t d0 = dig(kv0.x), d1 = dig(kv1.x);
        const OutRec in0 = s_out[d0];
        const OutRec in1 = s_out[d1];
        store_quad(L0, q0, kv0, vv0, in0, d0);
        if (two) store_quad(L1, q1, kv1, vv1, in1, d1);
    };

    // CL = 2 with split digits: the few-bucket ranking (launch_scatter picks it for nsplit < 4)
    constexpr bool FEW = DMODE == kDigitSplit && CL == 2;
    static_assert(CL != 2 || FEW, "CL = 2: split digits only");
    uint32_t hotd = 0xFFFFFFFFu;  // CL: the wave's last aggregated digit (none yet)
    uint32_t order_bad = 0;       // the per-tile rank check (rank_check) failed in this thread

    for (uint64_t tb = cbeg, tno = 0; tb < cend; tb += T, ++tno) {
        // the rank check on every kRankCheckEvery-th tile of a chunk, its first included (workgroup-uniform)
        const bool check_tile = (tno & (kRankCheckEvery - 1)) == 0;
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        const bool full = valid == T && head == 0;
        const uint64_t nb = tb + T;
        uint32_t plim = valid > base ? valid - base : 0u;  // slot j is real iff j * 64 < plim
        asm volatile("" : "+v"(plim));
        // ... and, in slot 0, iff this lane's tile position is not before the chunk (head)
        const bool h0 = base >= head;
        head = 0;
        // ---- 1. per-wave digit histogram (each wave clears its own counters first)
#pragma unroll
        for (uint32_t i = lane; i < R; i += kWave) s_cnt[w * RS + i] = 0;
        // rank first: the returning add IS the key's rank among its wave's keys of that digit
        // (lane order, kRankAtomic); two ranks (< 2^16) per register
        uint32_t rk[(KPT + 1) / 2];
        // split digits (a compare per splitter) are kept from step 1, 4 bits each, for step 3
        constexpr bool PD = DMODE == kDigitSplit && BITS <= 4;
        uint32_t dpk[PD ? (KPT + 7) / 8 : 1];
#pragma unroll
        for (int i = 0; i < (PD ? (KPT + 7) / 8 : 1); ++i) dpk[i] = 0;
        uint32_t nkey[KPT];
        uint32_t nval[PAIRS ? KPT : 1];
        constexpr int DB = CL ? hooks::kDeferKeysCl : hooks::kDeferKeysPlain;
        if (full && DB > 0 && !PD) {
            // deferred ranking: batches of DB slots issue their adds, then turn the returns into ranks
            static_assert(DB == 0 || KPT % (DB > 0 ? DB : 1) == 0, "whole batches");
#pragma unroll
            for (int j0 = 0; j0 < KPT; j0 += (DB > 0 ? DB : 1)) {
                uint32_t o[DB > 0 ? DB : 1], cc[DB > 0 ? DB : 1];
                uint64_t mm[DB > 0 ? DB : 1];
#pragma unroll
                for (int u = 0; u < DB; ++u)
                    o[u] = hot_issue<CL != 0>(&s_cnt[w * RS], dig(key[j0 + u]), hotd, cc[u], mm[u]);
#pragma unroll
                for (int u = 0; u < DB; ++u) {
                    const int j = j0 + u;
                    uint32_t r = hot_rank(o[u], dig(key[j]), cc[u], mm[u]);
                    if (j == 0 && check_tile) order_bad |= rank_check<BITS>(dig(key[j]), r, a.rank_fault);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            }
        } else if (full && FEW) {
            // partitions into <= 4 buckets (CL = 2, launch_scatter): 16-32 lanes of a slot share each digit,
            // and lane-ordered adds serialised them on one LDS counter (2^30 keys into 2 buckets: 2.8 ms
            // against 1.8 for 8). Here the wave's running count of each digit is a wave-uniform register:
            // a key's rank is its digit's count plus the lanes below with the same digit (one ballot per
            // digit); the counts go to the wave's counter row after the tile
            uint32_t c4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t dj = dig(key[j]);
                if constexpr (PD) dpk[j / 8] |= dj << (4 * (j % 8));
                uint32_t r = 0;
#pragma unroll
                for (uint32_t v = 0; v < 4; ++v) {
                    const uint64_t m = __ballot(dj == v);
                    if (dj == v)
                        r = c4[v] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    c4[v] += wave_count(m);
                }
                if (j == 0 && check_tile) order_bad |= rank_check<BITS>(dj, r, a.rank_fault);
                rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
            }
            if (lane < 4u) s_cnt[w * RS + lane] = lane == 0u ? c4[0] : lane == 1u ? c4[1] : lane == 2u ? c4[2] : c4[3];
        } else if (full) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                // (measured: rank_add's aggregation is ~2% faster than plain lane-ordered adds even
                // on uniform keys, 1.7x on clustered ones; dev/lines_exp.hip "rank1" +4% uniform)
                const uint32_t dj = dig(key[j]);
                if constexpr (PD) dpk[j / 8] |= dj << (4 * (j % 8));
                uint32_t r = CL ? rank_add_hot(&s_cnt[w * RS], dj, hotd) : rank_add(&s_cnt[w * RS], dj);
                if (j == 0 && check_tile) order_bad |= rank_check<BITS>(dj, r, a.rank_fault);
                rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
            }
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = dig(key[j]);
                if constexpr (PD) dpk[j / 8] |= d << (4 * (j % 8));
                uint32_t r = 0;
                if ((uint32_t)(j * kWave) < plim && (j != 0 || h0)) r = atomicAdd(&s_cnt[w * RS + d], 1u);
                rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
            }
        }
        // next tile's keys: in flight through the scan, staging and output phases
        if (nb < cend) load_tile(nb, nkey, nval);
        __syncthreads();

        // ---- 2. segments, line records, carry copy, counter bases
        // the group's TPD threads split the W per-wave counters of digit d; the leader combines
        constexpr uint32_t WPT = (W >= (int)TPD) ? W / TPD : 1;   // waves per group thread
        uint32_t part = 0;
        uint32_t wx[WPT];
        if (sub < (uint32_t)W) {
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i) {
                const uint32_t v = sub * WPT + i;
                wx[i] = v < (uint32_t)W ? s_cnt[v * RS + d_own] : 0u;
                part += wx[i];
            }
        }
        // exclusive prefix of the parts inside the group and the digit's tile count (the group is
        // TPD consecutive lanes of one wave)
        uint32_t gpre, cnt;
        group_scan<TPD>(part, sub, gpre, cnt);
        uint32_t wcnt = 0, A = 0, e = 0;
        if (leader) {
            A = g_run - carry;  // line-aligned
            e = g_run + cnt;
            wcnt = max(A, e & ~(uint32_t)(G - 1)) - A;  // whole lines only
        }
        uint32_t nseg;
        const uint32_t S = block_excl_scan1<THREADS>(wcnt, s_ws, nseg);  // next s_ws write is a tile later
        const uint32_t gS = group_lane<TPD>(S, 0), gw = group_lane<TPD>(wcnt, 0);
        const uint32_t gA = group_lane<TPD>(A, 0), gc = group_lane<TPD>(carry, 0), ginv = group_lane<TPD>(inv, 0);
        {
            const uint32_t d = d_own;
            // per-wave counter bases: after the carry, waves in order
            if (sub < (uint32_t)W) {
                uint32_t acc = gS + gc + gpre;
#pragma unroll
                for (uint32_t i = 0; i < WPT; ++i) {
                    const uint32_t v = sub * WPT + i;
                    if (v < (uint32_t)W) {
                        // {LDS base | the digit's line limit << 16} (both < CAP < 2^16), read back
                        // with one ds_read_b32 per key in step 3
                        s_cnt[v * RS + d] = acc | ((gS + gw) << 16);
                    }
                    acc += wx[i];
                }
            }
            // old carry -> segment head (only when a line is written; else it stays and grows)
            constexpr uint32_t CB = G / TPD;  // contiguous carry slots per group thread
            if constexpr (G % TPD == 0 && CB % 2 == 0) {
                // each thread moves its CB slots as 8-B pairs (the carry area and the segment head
                // are both line-aligned); only the pair holding the carry's end is split. 8-B LDS
                // stores, not 16-B ones: ds_write_b128 costs 13 cycles against 6 for b64
                // (MI355X_MICROARCH.md LDS table); dev/lines_exp.hip COPY64 -1 % per C3 pass
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                const uint32_t x0 = sub * CB;
                if (gw > 0 && x0 < gc) {
                    u32x2 ck[CB / 2], cv[PAIRS ? CB / 2 : 1];
#pragma unroll
                    for (uint32_t i = 0; i < CB / 2; ++i) {
                        ck[i] = *reinterpret_cast<const u32x2 *>(&s_stage[CAP + d * G + x0 + 2 * i]);
                        if constexpr (PAIRS) cv[i] = *reinterpret_cast<const u32x2 *>(&s_vstage[CAP + d * G + x0 + 2 * i]);
                    }
#pragma unroll
                    for (uint32_t i = 0; i < CB / 2; ++i) {
                        const uint32_t x = x0 + 2 * i;
                        if (x + 2 <= gc) {
                            *reinterpret_cast<u32x2 *>(&s_stage[gS + x]) = ck[i];
                            if constexpr (PAIRS) *reinterpret_cast<u32x2 *>(&s_vstage[gS + x]) = cv[i];
                        } else if (x < gc) {
                            s_stage[gS + x] = ck[i][0];
                            if constexpr (PAIRS) s_vstage[gS + x] = cv[i][0];
                        }
                    }
                }
            } else if (gw > 0) {
                // at most (G - 1 + TPD - 1) / TPD slots per thread: all reads, then all writes
                constexpr uint32_t CPT = (G - 1 + TPD - 1) / TPD;
                uint32_t ck[CPT], cv[PAIRS ? CPT : 1];
#pragma unroll
                for (uint32_t i = 0; i < CPT; ++i) {
                    const uint32_t x = sub + i * TPD;
                    if (x < gc) {
                        ck[i] = s_stage[CAP + d * G + x];
                        if constexpr (PAIRS) cv[i] = s_vstage[CAP + d * G + x];
                    }
                }
#pragma unroll
                for (uint32_t i = 0; i < CPT; ++i) {
                    const uint32_t x = sub + i * TPD;
                    if (x < gc) {
                        s_stage[gS + x] = ck[i];
                        if constexpr (PAIRS) s_vstage[gS + x] = cv[i];
                    }
                }
            }
            if (leader) {
                if constexpr (NX) s_out[d] = make_uint4(gA - gS, ((gS / G) << 8) | ginv, nb_own, 0u);
                else s_out[d] = make_uint2(gA - gS, ((gS / G) << 8) | ginv);
                if (gw > 0) inv = 0;
                carry = e - (A + gw);  // pending - written
                g_run = e;
                if (nb >= cend) s_flush[d] = make_uint2(g_run - carry, inv | (carry << 8));
            }
        }
        __syncthreads();

        // ---- 3. rank (lane-ordered returning LDS add) and stage; tails go to the carry.
        // Batches of 8 slots: all atomics and limit reads are issued before the first store,
        // so the LDS round trips overlap instead of serialising slot by slot.
        constexpr int SB = KPT < 8 ? KPT : 8;
        static_assert(KPT % SB == 0, "whole batches of slots");
#pragma unroll
        for (int j0 = 0; j0 < KPT; j0 += SB) {
            uint32_t pp[SB], ll[SB], dd[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                asm volatile("" : "+v"(key[j]));  // recompute: CSE with step 1 would pin KPT digits
                if constexpr (PD) dd[u] = (dpk[j / 8] >> (4 * (j % 8))) & 15u;
                else dd[u] = dig(key[j]);
                const uint32_t bl = s_cnt[w * RS + dd[u]];
                pp[u] = (bl & 0xFFFFu) + ((j & 1) ? (rk[j / 2] >> 16) : (rk[j / 2] & 0xFFFFu));
                ll[u] = bl >> 16;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                uint32_t idx = pp[u] < ll[u] ? pp[u] : CAP + dd[u] * G + (pp[u] - ll[u]);
                if (!(full || ((uint32_t)(j * kWave) < plim && (j != 0 || h0)))) idx = CAP + R * G;  // scratch slot
                s_stage[idx] = key[j];
                if constexpr (PAIRS) s_vstage[idx] = val[j];
            }
        }
        __syncthreads();

        // ---- 4. whole lines out: 4 keys per lane (16-B aligned in LDS and in global memory)
        const uint32_t nq = (nseg / G) * QPL;
        for (uint32_t item = t; item < nq; item += 2 * THREADS) out_pair(item, nq);
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            key[j] = nkey[j];
            if constexpr (PAIRS) val[j] = nval[j];
        }
    }
    // ---- chunk end: the carries (written by the last tile's staging, behind its barrier)
    if (cbeg < cend) {
        for (uint32_t item = t; item < R * G; item += THREADS) {
            const uint2 fl = s_flush[item / G];
            const uint32_t x = item % G;
            if ((fl.y & 0xFFu) <= x && x < (fl.y >> 8)) {
                const uint32_t k = s_stage[CAP + item];
                hooks::store_word(a.kout + (uint64_t)fl.x + x, k);
                if constexpr (PAIRS) hooks::store_word(a.vout + (uint64_t)fl.x + x, s_vstage[CAP + item]);
                if constexpr (NX) {
                    const uint32_t d = item / G;
                    if (count_next) next_add(d, fl.x + x - a.pos_shift >= s_nb[d] ? 1u : 0u, k);
                }
            }
        }
    }
    if constexpr (NX) {
        if (count_next) {
            __syncthreads();
            for (uint32_t i = t; i < 2 * R * R; i += THREADS) {
                uint32_t v = 0;
#pragma unroll
                for (uint32_t r = 0; r < NXR; ++r) v += s_next[i * NXR + r];
                if (v) {
                    const uint32_t d = i / (2 * R), slot = (i / R) % 2, e = i % R;
                    atomicAdd(&a.next_table[(uint64_t)e * a.num_chunks + s_oc[d] + slot], v);
                }
            }
            // the last workgroup scans the next pass's table (no scan launches between passes),
            // unless the next pass derives its offsets from the raw counts itself (raw_table)
            if (a.done != nullptr && a.tail_zero != nullptr) {
                __shared__ uint32_t s_last;
                tail_scan<THREADS>(a.next_table, (uint64_t)R * a.num_chunks, a.tail_zero, a.done, s_ws, &s_last,
                                   (uint32_t)a.n);
            }
        }
    }
    report_order(a.check, order_bad);
    RS_WG_T1;
}


// ------------------------------------------------------------------------------ scatter (pairs, 128-B lines)
// rs_scatter_pairs: the pass of rs_scatter_lines for key + value pairs with whole 128-B lines in BOTH
// output arrays (G = 32 keys). rs_scatter_lines' layout cannot do that for pairs: its LDS lines map
// one to one to global lines (every digit's segment starts on a line, T + 31R slots per array) and
// the carries live in an LDS area of their own (32R slots per array): 2 x (T + 63R) x 4 B = 190 KB at
// 8192-pair tiles, so pairs wrote 64-B lines (whose HBM floor is 1.3x that of 128-B lines,
// dev/runlen_lab.hip: 3.74 vs 2.90 ms per 2^30 pairs). Here:
//   * a digit's segment starts on a 16-B quad (not a line), so it wastes <= 3 slots, and it holds
//     carry + this tile's keys INCLUDING the tail past the last whole line: <= T + 34R slots per array;
//   * the tail goes back to REGISTERS (the digit's TPD threads hold 32 / TPD carry slots of keys
//     and values each) and is written into the next tile's segment head in step 2: no carry area;
//   * the output phase walks whole lines in order; a line's digit is the last digit whose first line
//     is at or before it (one bit per line start in a bitmap + the digit at each start), its LDS and
//     global positions the digit's record {global, LDS} + 32 x line.
// 2 x (8192 + 34 x 256 + 36) x 4 B = 135 KB + counters + records: fits 160 KB beside 8192-pair tiles.
// Per tile:
//   1. per-wave digit histogram with returning adds = ranks (as rs_scatter_lines)
//   2. segments (quad-aligned, packed with the whole-line count into one block scan), per-(wave,
//      digit) LDS bases, the carry written from registers into the segment head, line marks
//   3. stage keys and values at base + rank (tails included, no limit test)
//   4. whole lines out (8 lanes x 16 B per array per line), the tails read back into registers
// A chunk starts with `inv` invalid leading slots per digit (its first line begins before the
// chunk's output) and ends with masked dword stores of the carries (both lines are shared with the
// neighbouring chunks). Digit-group chunks (a.bounds) and the clustered-input ranking (CL) as in
// rs_scatter_lines. (The measured variants of this kernel -- two tiles of loads in flight, interleaved or
// sequential staging, deferred output, other load points -- are dev/pairs_variants.hpp.)
template <int BITS, int THREADS, int KPT, int CL = 0>
__global__ __launch_bounds__(THREADS, 1) void rs_scatter_pairs(ScatterArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int SEG = kWave * KPT;
    constexpr uint32_t T = THREADS * KPT;
    constexpr uint32_t G = 32;                       // keys per 128-B line
    constexpr uint32_t QPL = G / 4;                  // 16-B quads per line
    constexpr uint32_t TPD = THREADS / R;            // threads per digit
    constexpr uint32_t CPT = G / TPD;                // carry slots held per group thread
    constexpr uint32_t CAP = T + (G - 1) * R + 3 * R;  // staged slots, worst case
    constexpr uint32_t NLM = (T + (G - 1) * R) / G;    // whole lines per tile, worst case
    constexpr uint32_t NBW = (NLM + 31) / 32;          // bitmap words
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    static_assert(R <= THREADS && TPD <= kWave && CPT % 4 == 0, "a digit's group in one wave, whole carry quads");
    static_assert(CAP + 40 < 65536u && NLM < 65536u, "slot and line indices packed in 16 bits");

    // [0, CAP) segments; [CAP, CAP + 32) the last tail read's overrun; CAP + 32 the padding sink
    __shared__ __attribute__((aligned(16))) uint32_t s_k[CAP + 36];
    __shared__ __attribute__((aligned(16))) uint32_t s_v[CAP + 36];
    constexpr uint32_t RS = counter_stride<R, TPD, (W >= (int)TPD) ? W / TPD : 0>();
    __shared__ uint32_t s_cnt[W * RS + 1];
    __shared__ uint4 s_rec[R];        // per digit: {global - 32 x first line, LDS - 32 x first line, first line << 8 | inv}
    __shared__ uint8_t s_mark[NLM + 1];  // digit of the line that starts a digit's lines
    __shared__ uint32_t s_bits[NBW];     // line starts
    __shared__ uint2 s_lrec[NLM];        // per whole line: {global key index, LDS index | inv << 16}
    __shared__ uint32_t s_ws[W];

    const uint32_t t = threadIdx.x;
    const uint32_t w = t / kWave;
    const uint32_t lane = lane_id();
    const uint32_t c = blockIdx.x;
    const Digit<BITS, kDigitShift> dig{a.shift, 0, nullptr};
    uint64_t cbeg = (uint64_t)c * a.chunk_keys;
    uint64_t cend = min(cbeg + a.chunk_keys, a.n);
    uint32_t head = 0;
    if (a.cl_select != nullptr && ((*a.cl_select != kGroupsWhole) != (CL != 0))) return;
    if (a.bounds != nullptr && a.bounds[0] != 0u) {
        const uint64_t b = a.bounds[1 + c];
        cend = a.bounds[2 + c];
        cbeg = b < cend ? (b & ~(uint64_t)(kWave - 1)) : cend;
        head = (uint32_t)(b < cend ? b - cbeg : 0);
    }

    const uint32_t d_own = t / TPD;
    const uint32_t sub = t % TPD;
    const bool leader = sub == 0;
    // group state (the same in every thread of the group): running global position, carry length,
    // invalid leading slots of the chunk's first line; carry slots sub * CPT .. + CPT - 1 in ck / cv
    uint32_t g_run, carry, inv;
    {
        const uint32_t g = a.table[(uint64_t)d_own * a.num_chunks + c] + a.pos_shift;  // (as rs_scatter_lines)
        carry = g & (G - 1u);
        inv = carry;
        g_run = g;
    }
    uint32_t ck[CPT], cv[CPT];
#pragma unroll
    for (uint32_t i = 0; i < CPT; ++i) ck[i] = cv[i] = 0u;

    const uint32_t base = w * SEG + lane;
    auto load_tile = [&](uint64_t tb, uint32_t (&k)[KPT], uint32_t (&v)[KPT]) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        uint32_t lb = base;
        asm volatile("" : "+v"(lb));
        const uint32_t *__restrict__ tk = a.kin + tb + lb;
        const uint32_t *__restrict__ tv = a.vin + tb + lb;
        if (valid == T) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                k[j] = tk[j * kWave];
                v[j] = tv[j * kWave];
            }
        } else {
            const uint32_t lim = valid > lb ? valid - lb : 0u;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool in = (uint32_t)(j * kWave) < lim;
                k[j] = in ? tk[j * kWave] : 0u;
                v[j] = in ? tv[j * kWave] : 0u;
            }
        }
    };

    // the digit of whole line V: the last marked line start at or before V
    auto line_digit = [&](uint32_t V) {
        uint32_t wi = V >> 5;
        uint32_t m = s_bits[wi] & (0xFFFFFFFFu >> (31u - (V & 31u)));
        while (m == 0u) m = s_bits[--wi];  // (line 0 is always marked)
        return (uint32_t)s_mark[wi * 32u + 31u - (uint32_t)__builtin_clz(m)];
    };
    auto store_item = [&](uint32_t item) {
        const uint32_t V = item / QPL, q = (item % QPL) * 4u;
        const uint2 lr = s_lrec[V];
        const uint32_t li = (lr.y & 0xFFFFu) + q;
        const u32x4 kv = *reinterpret_cast<const u32x4 *>(&s_k[li]);
        const u32x4 vv = *reinterpret_cast<const u32x4 *>(&s_v[li]);
        const uint64_t gp = (uint64_t)(lr.x + q);
        const uint32_t lo = lr.y >> 16;
        if (lo <= q) {
            hooks::store_quad_nt(a.kout + gp, kv);
            hooks::store_quad_nt(a.vout + gp, vv);
        } else {
            // the chunk's first line of this digit: lanes below lo belong to the previous chunk
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x)
                if (lo <= q + x) {
                    hooks::store_word(a.kout + gp + x, kv[x]);
                    hooks::store_word(a.vout + gp + x, vv[x]);
                }
        }
    };

    RS_STAMP_DECL
    // ---- 4. (of a tile) the tails back into the carry registers (the quads holding any); whole lines out
    auto output = [&](const uint32_t S, const uint32_t wl, const uint32_t pending, const uint32_t nlines,
                      const uint32_t cnt) {
        {
            const uint32_t tl0 = S + wl * G + sub * CPT;  // quad-aligned
            const uint32_t ncarry = pending - wl * G;
#pragma unroll
            for (uint32_t i = 0; i < CPT; i += 4) {
                if (sub * CPT + i >= ncarry) break;
                const u32x4 kq = *reinterpret_cast<const u32x4 *>(&s_k[tl0 + i]);
                const u32x4 vq = *reinterpret_cast<const u32x4 *>(&s_v[tl0 + i]);
                ck[i] = kq.x; ck[i + 1] = kq.y; ck[i + 2] = kq.z; ck[i + 3] = kq.w;
                cv[i] = vq.x; cv[i + 1] = vq.y; cv[i + 2] = vq.z; cv[i + 3] = vq.w;
            }
        }
        const uint32_t nq = nlines * QPL;
        for (uint32_t item = t; item < nq; item += 2 * THREADS) {
            store_item(item);
            if (item + THREADS < nq) store_item(item + THREADS);
        }
        RS_STAMP(4);
        if (wl > 0) inv = 0;
        carry = pending - wl * G;
        g_run += cnt;
    };

    uint32_t hotd = 0xFFFFFFFFu;
    uint32_t order_bad = 0;  // the per-tile rank check (rank_check) failed in this thread
    uint32_t key[KPT], val[KPT];
    if (cbeg < cend) load_tile(cbeg, key, val);
    for (uint64_t tb = cbeg, tno = 0; tb < cend; tb += T, ++tno) {
        // the rank check on every kRankCheckEvery-th tile of a chunk, its first included (workgroup-uniform)
        const bool check_tile = (tno & (kRankCheckEvery - 1)) == 0;
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        const bool full = valid == T && head == 0;
        const uint64_t nb = tb + T;
        uint32_t plim = valid > base ? valid - base : 0u;
        asm volatile("" : "+v"(plim));
        const bool h0 = base >= head;
        head = 0;
        // ---- 1. per-wave digit histogram; the returning add is the key's rank among its wave's
        //      keys of that digit (lane order, kRankAtomic); two ranks per register
#pragma unroll
        for (uint32_t i = lane; i < R; i += kWave) s_cnt[w * RS + i] = 0;
        uint32_t rk[(KPT + 1) / 2];
        uint32_t nkey[KPT], nval[KPT];
        constexpr int DB = hooks::kDeferPairs;
        if (full && DB > 0) {
            // deferred ranking (hot_issue / hot_rank): the slots' adds back to back, one LDS wait
            // per batch of DB slots (C4: 3.45 vs 3.48 ms per pass, dev/lab.sh ab)
            static_assert(DB == 0 || KPT % (DB > 0 ? DB : 1) == 0, "whole batches");
#pragma unroll
            for (int j0 = 0; j0 < KPT; j0 += (DB > 0 ? DB : 1)) {
                uint32_t o[DB > 0 ? DB : 1], cc[DB > 0 ? DB : 1];
                uint64_t mm[DB > 0 ? DB : 1];
#pragma unroll
                for (int u = 0; u < DB; ++u)
                    o[u] = hot_issue<CL != 0>(&s_cnt[w * RS], dig(key[j0 + u]), hotd, cc[u], mm[u]);
#pragma unroll
                for (int u = 0; u < DB; ++u) {
                    const int j = j0 + u;
                    uint32_t r = hot_rank(o[u], dig(key[j]), cc[u], mm[u]);
                    if (j == 0 && check_tile) order_bad |= rank_check<BITS>(dig(key[j]), r, a.rank_fault);
                    rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                }
            }
        } else if (full) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t dj = dig(key[j]);
                uint32_t r = CL ? rank_add_hot(&s_cnt[w * RS], dj, hotd) : rank_add(&s_cnt[w * RS], dj);
                if (j == 0 && check_tile) order_bad |= rank_check<BITS>(dj, r, a.rank_fault);
                rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
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
        RS_STAMP(5);
        // the next tile's loads: in flight through steps 2-4 (issued earlier or later measured slower,
        // dev/pairs_variants.hpp)
        if (nb < cend) load_tile(nb, nkey, nval);
        // (the previous tile's step 4 has read the bitmap, records and staging area: behind the
        // barrier below)
        __syncthreads();
        RS_STAMP(0);

        // ---- 2. segments, bases, carry in, line marks
        constexpr uint32_t WPT = (W >= (int)TPD) ? W / TPD : 1;
        uint32_t part = 0;
        uint32_t wx[WPT];
        if (sub < (uint32_t)W) {
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i) {
                const uint32_t v = sub * WPT + i;
                wx[i] = v < (uint32_t)W ? s_cnt[v * RS + d_own] : 0u;
                part += wx[i];
            }
        }
        uint32_t gpre, cnt;
        group_scan<TPD>(part, sub, gpre, cnt);
        // (carry, g_run, inv are the same in every thread of the group)
        const uint32_t A = g_run - carry;          // line-aligned
        const uint32_t pending = carry + cnt;      // slots from A on
        const uint32_t wl = pending / G;           // whole lines written this tile
        const uint32_t seg = (pending + 3u) & ~3u;
        if (t < NBW) s_bits[t] = 0u;
        uint32_t tot;
        const uint32_t pre = block_excl_scan1<THREADS>(leader ? (seg | (wl << 16)) : 0u, s_ws, tot);
        RS_STAMP(7);
        const uint32_t S = group_lane<TPD>(pre, 0) & 0xFFFFu, LS = group_lane<TPD>(pre, 0) >> 16;
        const uint32_t nlines = tot >> 16;
        if (sub < (uint32_t)W) {
            uint32_t acc = S + carry + gpre;
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i) {
                const uint32_t v = sub * WPT + i;
                if (v < (uint32_t)W) s_cnt[v * RS + d_own] = acc;
                acc += wx[i];
            }
        }
        // the carry from registers into the segment head, whole quads (a quad past the carry's end
        // lies inside the segment and is overwritten by step 3)
#pragma unroll
        for (uint32_t i = 0; i < CPT; i += 4) {
            if (sub * CPT + i < carry) {
                *reinterpret_cast<u32x4 *>(&s_k[S + sub * CPT + i]) = u32x4{ck[i], ck[i + 1], ck[i + 2], ck[i + 3]};
                *reinterpret_cast<u32x4 *>(&s_v[S + sub * CPT + i]) = u32x4{cv[i], cv[i + 1], cv[i + 2], cv[i + 3]};
            }
        }
        if (leader) {
            s_rec[d_own] = make_uint4(A - LS * G, S - LS * G, (LS << 8) | inv, 0u);
            if (wl > 0) {
                s_mark[LS] = (uint8_t)d_own;
                atomicOr(&s_bits[LS >> 5], 1u << (LS & 31u));
            }
        }
        RS_STAMP(6);
        __syncthreads();
        RS_STAMP(1);

        // ---- 3. each whole line's record (its digit from the bitmap: one lookup per line here
        //      instead of a dependent chain per quad in step 4); stage every slot at base + rank
        //      (batches of 8: all reads before the stores)
        for (uint32_t V = t; V < nlines; V += THREADS) {
            const uint4 rec = s_rec[line_digit(V)];
            const uint32_t lo = (rec.z >> 8) == V ? (rec.z & 0xFFu) : 0u;
            s_lrec[V] = make_uint2(rec.x + V * G, (rec.y + V * G) | (lo << 16));
        }
        RS_STAMP(2);
        constexpr int SB = KPT < 8 ? KPT : 8;
        static_assert(KPT % SB == 0, "whole batches of slots");
#pragma unroll
        for (int j0 = 0; j0 < KPT; j0 += SB) {
            uint32_t pp[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                asm volatile("" : "+v"(key[j]));
                pp[u] = s_cnt[w * RS + dig(key[j])] + ((j & 1) ? (rk[j / 2] >> 16) : (rk[j / 2] & 0xFFFFu));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int j = j0 + u;
                uint32_t idx = pp[u];
                if (!(full || ((uint32_t)(j * kWave) < plim && (j != 0 || h0)))) idx = CAP + 32;  // sink
                s_k[idx] = key[j];
                s_v[idx] = val[j];
            }
        }
        __syncthreads();
        RS_STAMP(3);

        output(S, wl, pending, nlines, cnt);
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            key[j] = nkey[j];
            val[j] = nval[j];
        }
    }
    // ---- chunk end: the carries (slots inv .. carry - 1 from the line at g_run - carry)
    if (cbeg < cend) {
        const uint64_t A = (uint64_t)(g_run - carry);
#pragma unroll
        for (uint32_t i = 0; i < CPT; ++i) {
            const uint32_t x = sub * CPT + i;
            if (x >= inv && x < carry) {
                hooks::store_word(a.kout + A + x, ck[i]);
                hooks::store_word(a.vout + A + x, cv[i]);
            }
        }
    }
    report_order(a.check, order_bad);
    RS_STAMP_FLUSH();
}

// Top-bits histogram of every stride-th 256-key block (the multi-GPU sort's splitter sample):
// 1024 threads take four sampled blocks per iteration into 2^top_bits LDS counters, then add
// them into the zeroed hist (one workgroup per CU keeps that final add to 2^top_bits per CU).
__global__ __launch_bounds__(1024) void rs_top_hist_sampled(const uint32_t *keys, uint64_t n, uint32_t top_bits,
                                                            uint32_t stride, uint32_t *hist) {
    __shared__ uint32_t s_h[1u << 12];
    const uint32_t t = threadIdx.x;
    const uint32_t bins = 1u << top_bits;
    for (uint32_t i = t; i < bins; i += 1024) s_h[i] = 0;
    __syncthreads();
    const uint64_t nsb = ((n + 255) / 256 + stride - 1) / stride;  // sampled blocks
    for (uint64_t sb = (uint64_t)blockIdx.x * 4 + t / 256; sb < nsb; sb += (uint64_t)gridDim.x * 4) {
        const uint64_t i = sb * stride * 256 + (t % 256);
        if (i < n) count_add(s_h, keys[i] >> (32 - top_bits));
    }
    __syncthreads();
    for (uint32_t i = t; i < bins; i += 1024)
        if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// The multi-GPU sort's splitter sample (rsort_multi_sample_plan): out[j] = keys[min(n - 1, j * stride +
// stride / 2)] for j < count, padded with 0xFFFFFFFF up to row_len (the padding sorts last).
__global__ void rs_sample(const uint32_t *keys, uint64_t n, uint64_t stride, uint64_t count, uint64_t row_len,
                          uint32_t *out) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < row_len; j += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0xFFFFFFFFu;
        if (j < count && n > 0) v = keys[min(n - 1, j * stride + stride / 2)];
        out[j] = v;
    }
}

__global__ void rs_gather_starts(const uint32_t *table, uint32_t num_chunks, uint32_t bins,
                                 uint64_t n, uint32_t *starts) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < bins) starts[d] = table[(uint64_t)d * num_chunks];
    if (d == bins) starts[d] = (uint32_t)n;
}

__global__ void rs_diff_starts(const uint32_t *starts, uint32_t bins, uint32_t *hist) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < bins) hist[d] = starts[d + 1] - starts[d];
}

__global__ void rs_widen(const uint32_t *in, unsigned long long *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Order-independent fingerprint of a key (or key + value) multiset and the count of adjacent
// descents: out[0] += sum of fmix64(value << 32 | key), out[1] += #{i : keys[i] > keys[i + 1]}.
// A sorted permutation of the input has the input's out[0] and out[1] == 0 (bench.py's check
// of the timed output; rsort_fingerprint_device).
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

__global__ __launch_bounds__(256) void rs_fingerprint(const uint32_t *keys, const uint32_t *vals, uint64_t n,
                                                      unsigned long long *out) {
    uint64_t h = 0, desc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        const uint64_t v = vals ? vals[i] : 0u;
        h += fmix64((v << 32) | k);
        if (i + 1 < n && k > keys[i + 1]) ++desc;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        h += (uint64_t)__shfl_xor((unsigned long long)h, o);
        desc += (uint64_t)__shfl_xor((unsigned long long)desc, o);
    }
    if (lane_id() == 0) {
        atomicAdd(&out[0], (unsigned long long)h);
        if (desc) atomicAdd(&out[1], (unsigned long long)desc);
    }
}

__global__ void rs_gen_uniform(uint32_t *out, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)(splitmix64(seed + i) >> 32);
}

__global__ void rs_gen_zipf(uint32_t *out, uint64_t n, uint64_t seed, const uint32_t *cdf,
                            uint64_t ranks) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)(splitmix64(seed + i) >> 32);
        uint64_t lo = 0, hi = ranks;  // first r with cdf[r] >= u
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cdf[mid] < u) lo = mid + 1; else hi = mid;
        }
        if (lo >= ranks) lo = ranks - 1;
        out[i] = fmix32((uint32_t)lo);
    }
}

__global__ void rs_gen_iota(uint32_t *out, uint64_t n, uint32_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = base + (uint32_t)i;
}

// ------------------------------------------------------------------------------ dispatch
// Kernel pointers with their names recorded (rsort_scatter_kernels_used).
template <int BITS, int THREADS, int KPT, int G, bool PAIRS, int DMODE, int NT = 0, int CL = 0>
static void *reg_lines() {
    void *fn = reinterpret_cast<void *>(&rs_scatter_lines<BITS, THREADS, KPT, G, PAIRS, DMODE, NT, CL>);
    static const bool once = [fn] {
        char nm[96];
        snprintf(nm, sizeof nm, "rs_scatter_lines<%d, %d, %d, %d, %s, %d, %d, %d>", BITS, THREADS, KPT, G,
                 PAIRS ? "true" : "false", DMODE, NT, CL);
        register_kernel(fn, nm, true);
        return true;
    }();
    (void)once;
    return fn;
}

template <int BITS, int THREADS, int KPT, int CL = 0>
static void *reg_pairs() {
    void *fn = reinterpret_cast<void *>(&rs_scatter_pairs<BITS, THREADS, KPT, CL>);
    static const bool once = [fn] {
        char nm[96];
        snprintf(nm, sizeof nm, "rs_scatter_pairs<%d, %d, %d, %d>", BITS, THREADS, KPT, CL);
        register_kernel(fn, nm, true);
        return true;
    }();
    (void)once;
    return fn;
}

// Pairs with k = 7, 8 write 128-B lines through rs_scatter_pairs; RSORT_PAIRS64=1 under RSORT_LAB=1
// selects rs_scatter_lines' 64-B-line pairs kernel instead (A/B measurements, dev/lab.sh).
static bool pairs_lines64() {
    static const bool v = [] {
        const char *e = lab_env("RSORT_PAIRS64");
        return e != nullptr && e[0] != '\0' && e[0] != '0';
    }();
    return v;
}

template <int BITS, int THREADS, int KPT, bool PAIRS, int RANK, int DMODE, int MINW>
static void *reg_scatter() {
    void *fn = reinterpret_cast<void *>(&rs_scatter<BITS, THREADS, KPT, PAIRS, RANK, DMODE, MINW>);
    static const bool once = [fn] {
        char nm[96];
        snprintf(nm, sizeof nm, "rs_scatter<%d, %d, %d, %s, %d, %d, %d>", BITS, THREADS, KPT, PAIRS ? "true" : "false",
                 RANK, DMODE, MINW);
        register_kernel(fn, nm);
        return true;
    }();
    (void)once;
    return fn;
}

template <int BITS>
static hipError_t hist_bits(int dmode, const HistArgs &a, hipStream_t s) {
    if (dmode == kDigitSplit) {
        if constexpr (BITS <= 5) {
            rs_histogram<BITS, kHistThreads, kDigitSplit, 1, 8><<<a.num_chunks * a.split, kHistThreads, 0, s>>>(a);
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
    if (a.split > 1 || a.wide) {
        // few long chunks split over workgroups: 1024-thread workgroups read fastest
        // (dev/scatter_lab.hip "hist": 6.0 TB/s vs 5.6 TB/s for 256 threads)
        // non-temporal 16-B loads: 6.8 TB/s vs 6.1 TB/s; 8 sub-counters per digit: clustered
        // Zipf keys (every pass after the first) 1.58 -> 0.63 ms at 2^30 (dev/scatter_lab.hip)
        rs_histogram<BITS, 1024, kDigitShift, 1, 8><<<a.num_chunks * a.split, 1024, 0, s>>>(a);
        return hipGetLastError();
    }
    rs_histogram<BITS, kHistThreads, kDigitShift, 1, 8><<<a.num_chunks * a.split, kHistThreads, 0, s>>>(a);
    return hipGetLastError();
}

// The compiled scatter kernels. "match" (the default public rank algorithm) runs kRankAtomic, the
// lane-ordered returning LDS add per key (kRankCount, the ballot peer match, where the lane-order
// probe fails or RSORT_RANK_BALLOT asks for it); "split" is the reference's 1-bit split sort.
// Geometries per kGeomShape.
template <int BITS, bool PAIRS, int RANK, int DMODE, int G>
static void *scatter_fn() {
    constexpr int TH = kGeomShape[G].threads;
    constexpr int KPT = kGeomShape[G].kpt;
    constexpr int MINW = (G == kGeomK4) ? 4 : 0;
    return reg_scatter<BITS, TH, KPT, PAIRS, RANK, DMODE, MINW>();
}

// count-first ranking: rank = kRankAtomic (lane-ordered LDS adds) or kRankCount (ballots)
template <int BITS, bool PAIRS, int DMODE, int G>
static void *scatter_cf(int rank) {
    return rank == kRankAtomic ? scatter_fn<BITS, PAIRS, kRankAtomic, DMODE, G>()
                               : scatter_fn<BITS, PAIRS, kRankCount, DMODE, G>();
}

template <int BITS, bool PAIRS>
static void *scatter_pick2(int rank, int dmode, int geom, int aligned16) {
    if (rank != kRankSplit && rank != kRankAtomic && rank != kRankCount) return nullptr;
    if (dmode == kDigitSplit) {
        if constexpr (BITS <= 5) {
            if constexpr (BITS >= 2) {
                // partition into 3..32 key ranges: whole lines from 4096-key tiles, like k = 3, 4
                // (a digit's thread group must fit one wave: BITS >= 2)
                constexpr int TH = kGeomShape[kGeomSmall].threads, KP = kGeomShape[kGeomSmall].kpt;
                if (geom == kGeomSmall && rank == kRankAtomic && aligned16)
                    return reg_lines<BITS, TH, KP, PAIRS ? kLineKeysPairs : kLineKeys,
                                                                      PAIRS, kDigitSplit, PAIRS ? 2 : 3>();
            }
            if constexpr (BITS >= 3 && !PAIRS) {
                // keys-only partitions of large inputs: 8192-key tiles of 512 threads (kGeomK4's shape)
                constexpr int TH = kGeomShape[kGeomK4].threads, KP = kGeomShape[kGeomK4].kpt;
                if (geom == kGeomK4 && rank == kRankAtomic && aligned16)
                    return reg_lines<BITS, TH, KP, kLineKeys, false, kDigitSplit, 3>();
            }
            if (geom == kGeomSmall && rank != kRankSplit) return scatter_cf<BITS, PAIRS, kDigitSplit, kGeomSmall>(rank);
            if constexpr (BITS >= 3 && !PAIRS) {
                if (geom == kGeomK4 && rank != kRankSplit) return scatter_cf<BITS, false, kDigitSplit, kGeomK4>(rank);
            }
        }
        return nullptr;
    }
    if (rank == kRankSplit) {
        if (geom == kGeomSmall) return scatter_fn<BITS, PAIRS, kRankSplit, kDigitShift, kGeomSmall>();
        return nullptr;
    }
    if (geom == kGeomSmall) {
        if constexpr (BITS >= 3 && BITS <= 4 && !PAIRS) {
            // k = 3, 4 keys: whole 128-B lines from 4096-key tiles (lane-ordered atomics and 16-B
            // aligned outputs, like kGeomLines)
            constexpr int TH = kGeomShape[kGeomSmall].threads, KP = kGeomShape[kGeomSmall].kpt;
            if (rank == kRankAtomic && aligned16)
                return reg_lines<BITS, TH, KP, kLineKeys, false, kDigitShift, 3>();
        }
        return scatter_cf<BITS, PAIRS, kDigitShift, kGeomSmall>(rank);
    }
    if constexpr (BITS >= 4 && BITS <= 8) {
        if (geom == kGeomLarge) return scatter_cf<BITS, PAIRS, kDigitShift, kGeomLarge>(rank);
        // whole-line stores need lane-ordered atomics and 16-B aligned outputs; else the same
        // tiles through rs_scatter. Non-temporal (NT): keys-only loads and stores; pairs stores
        // only (dev/scatter_lab LAB_PAIRS, 2^30: 4.24 -> 3.96 ms; nt loads 4.66 ms)
        constexpr int GL = PAIRS ? kGeomLinesPairs : kGeomLines;
        if (geom == GL) {
            if constexpr (PAIRS && (kGeomShape[GL].threads >> BITS) <= 8) {  // (carry slots per thread >= 4)
                // rank_add_hot's ranking on every pass, uniform keys too: 3.51 vs 3.84 ms per 2^30-pair
                // pass with rank_add, 3.52 vs 3.78 on Zipf pass 0, 3.63 vs 3.80 on Zipf pass 1
                // (dev/pairs_lab.hip, round-robin best of 3); one kernel, no clustered twin
                if (rank == kRankAtomic && aligned16 && !pairs_lines64())
                    return reg_pairs<BITS, kGeomShape[GL].threads, kGeomShape[GL].kpt, 1>();
            }
            if (rank == kRankAtomic && aligned16)
                return reg_lines<BITS, kGeomShape[GL].threads, kGeomShape[GL].kpt,
                                                                  PAIRS ? kLineKeysPairs : kLineKeys, PAIRS,
                                                                  kDigitShift, PAIRS ? 2 : 3>();
            return scatter_cf<BITS, PAIRS, kDigitShift, GL>(rank);
        }
    }
    if constexpr (BITS <= 4 && !PAIRS) {
        if (geom == kGeomK4) return scatter_cf<BITS, PAIRS, kDigitShift, kGeomK4>(rank);
    }
    return nullptr;
}

// k = 13 (the reference's largest digit, Parallel7.cu:740-745): 128-thread 4096-key tiles, every ranking
template <bool PAIRS>
static void *scatter_pick13(int rank, int dmode, int geom) {
    if (dmode != kDigitShift || geom != kGeomXL) return nullptr;
    if (rank == kRankSplit) return scatter_fn<13, PAIRS, kRankSplit, kDigitShift, kGeomXL>();
    if (rank != kRankAtomic && rank != kRankCount) return nullptr;
    return scatter_cf<13, PAIRS, kDigitShift, kGeomXL>(rank);
}

template <int BITS>
static void *scatter_pick(int pairs, int rank, int dmode, int geom, int aligned16) {
    if constexpr (BITS == 13) return pairs ? scatter_pick13<true>(rank, dmode, geom) : scatter_pick13<false>(rank, dmode, geom);
    else return pairs ? scatter_pick2<BITS, true>(rank, dmode, geom, aligned16)
                 : scatter_pick2<BITS, false>(rank, dmode, geom, aligned16);
}

static void *scatter_kernel(int bits, int pairs, int rank, int dmode, int geom, int aligned16) {
    switch (bits) {
        case 1: return scatter_pick<1>(pairs, rank, dmode, geom, aligned16);
        case 2: return scatter_pick<2>(pairs, rank, dmode, geom, aligned16);
        case 3: return scatter_pick<3>(pairs, rank, dmode, geom, aligned16);
        case 4: return scatter_pick<4>(pairs, rank, dmode, geom, aligned16);
        case 5: return scatter_pick<5>(pairs, rank, dmode, geom, aligned16);
        case 6: return scatter_pick<6>(pairs, rank, dmode, geom, aligned16);
        case 7: return scatter_pick<7>(pairs, rank, dmode, geom, aligned16);
        case 8: return scatter_pick<8>(pairs, rank, dmode, geom, aligned16);
        case 9: return scatter_pick<9>(pairs, rank, dmode, geom, aligned16);
        case 10: return scatter_pick<10>(pairs, rank, dmode, geom, aligned16);
        case 11: return scatter_pick<11>(pairs, rank, dmode, geom, aligned16);
        case 12: return scatter_pick<12>(pairs, rank, dmode, geom, aligned16);
        case 13: return scatter_pick<13>(pairs, rank, dmode, geom, aligned16);
        default: return nullptr;
    }
}


// ------------------------------------------------------------------------------ lane-order probe
// The default ranking (kRankAtomic) rests on gfx950's LDS serving the lanes of one ds_add_rtn_u32
// that hit the same address in ascending lane order. The probe replays the production conditions of
// the line kernels: the 1024-thread shape of the k = 8 keys and pairs kernels (counter rows
// counter_stride = 260 words apart) and the 512-thread shape of the partition kernels (rows 264
// apart at 256 digits), the SAME device functions the kernels instantiate -- rank_add (any exec
// mask), rank_add_hot with its agg_add paths and the deferred hot_issue / hot_rank (full waves, as
// in the kernels' full tiles) -- on digit ranges 1..256, runs of equal digits (with several runs
// sharing a digit), a run crossing the slot, partial exec masks; and checks every
// returned rank against old value + #lower active lanes with the same digit (a register-only count).
// Any mismatch makes the library use ballots.
template <int THREADS>
__global__ __launch_bounds__(THREADS) void rs_lane_order_probe(uint32_t *bad) {
    constexpr uint32_t R = 256;
    constexpr int W = THREADS / kWave;
    constexpr uint32_t TPD = THREADS / R;
    constexpr uint32_t RS = counter_stride<R, TPD, (W >= (int)TPD) ? W / TPD : 0>();
    __shared__ uint32_t s_cnt[W * RS];
    const uint32_t t = threadIdx.x, w = t / kWave, lane = lane_id();
    for (uint32_t i = t; i < W * RS; i += THREADS) s_cnt[i] = 0;
    __syncthreads();
    uint32_t nbad = 0;
    uint32_t hot = 0xFFFFFFFFu;
    for (uint32_t it = 0; it < 192; ++it) {
        uint32_t h = (blockIdx.x * 0x9E3779B9u) ^ (it * 0x85EBCA6Bu) ^ (t * 0xC2B2AE35u);
        h ^= h >> 16;
        h *= 0x7feb352dU;
        h ^= h >> 15;
        const uint32_t hw = __builtin_amdgcn_readfirstlane((blockIdx.x * 0x27D4EB2Fu) ^ (it * 0x165667B1u) ^ w);
        const uint32_t L = 1u + hw % 37u;  // run length of the run patterns
        uint32_t d;
        switch (it % 8) {
            case 0: d = 0; break;                                     // one counter
            case 1: d = h % 3; break;
            case 2: d = h % 16; break;
            case 3: d = h % 256; break;                               // uniform keys
            case 4: d = (hw + lane / L) % 256; break;                 // runs of equal digits
            case 5: d = (lane < (hw % 64) ? hw : hw + 1 + (h & 1)) % 256; break;  // a run crossing the slot
            case 6: d = (hw + (lane / L) % 3) % 256; break;           // runs, several sharing a digit
            default: d = (hw + (lane / (1u + hw % 5u)) * 7u) % 256;   // many short runs (> 32: the fallback)
        }
        // which ranking: rank_add (partial exec masks too), rank_add_hot, and the deferred hot_issue +
        // hot_rank with and without the hot candidate (full waves, as in the kernels)
        const uint32_t fn = (it / 8) % 4;
        const bool active = fn != 0 || (it % 3 == 0) || ((h >> 7) % 4 != 0);
        const uint32_t before = s_cnt[w * RS + d];
        // #lower active lanes with the same digit, from registers only: the lanes whose 8 digit bits
        // all equal mine (8 ballots, every lane taking part), among the active ones
        uint64_t same = __ballot(active);
#pragma unroll
        for (uint32_t b = 0; b < 8; ++b) {
            const uint64_t ones = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? ones : ~ones;
        }
        const uint32_t below = (uint32_t)__popcll(same & lanes_below());
        __builtin_amdgcn_wave_barrier();
        if (active) {
            uint32_t got;
            if (fn == 0) {
                got = rank_add(&s_cnt[w * RS], d);
            } else if (fn == 1) {
                got = rank_add_hot(&s_cnt[w * RS], d, hot);
            } else {
                uint32_t c;
                uint64_t m;
                const uint32_t o = fn == 2 ? hot_issue<true>(&s_cnt[w * RS], d, hot, c, m)
                                           : hot_issue<false>(&s_cnt[w * RS], d, hot, c, m);
                got = hot_rank(o, d, c, m);
            }
            nbad += got != before + below;
        }
        __builtin_amdgcn_wave_barrier();
        if (it % 24 == 23) {  // keep the counters small (each wave clears its own row)
            for (uint32_t i = lane; i < R; i += kWave) s_cnt[w * RS + i] = 0;
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int lane_order_probe() {
    static std::mutex mu;
    static int state[64] = {0};  // per device: 0 unknown, 1 ordered, 2 not ordered
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    std::lock_guard<std::mutex> g(mu);
    if (state[dev]) return state[dev] == 1 ? 1 : 0;
    hipStream_t s = nullptr;
    uint32_t *bad = nullptr;
    uint32_t host = 1;
    bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&bad, 4) == hipSuccess && hipMemsetAsync(bad, 0, 4, s) == hipSuccess;
    if (ok) {
        rs_lane_order_probe<1024><<<512, 1024, 0, s>>>(bad);  // the k = 8 keys and pairs kernels' shape
        rs_lane_order_probe<512><<<512, 512, 0, s>>>(bad);    // 512-thread workgroups (partitions)
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(&host, bad, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
    }
    if (bad) (void)hipFree(bad);
    if (s) (void)hipStreamDestroy(s);
    if (!ok) return -1;
    state[dev] = host == 0 ? 1 : 2;
    return host == 0 ? 1 : 0;
}

int internal_rank(int public_algo) {
    if (public_algo == 1) return kRankSplit;   // RSORT_RANK_SPLIT
    if (public_algo == 2) return kRankCount;   // RSORT_RANK_BALLOT
    return lane_order_probe() == 1 ? kRankAtomic : kRankCount;
}

hipError_t launch_histogram(int bits, int dmode, const HistArgs &a, hipStream_t s) {
    switch (bits) {
        case 1: return hist_bits<1>(dmode, a, s);
        case 2: return hist_bits<2>(dmode, a, s);
        case 3: return hist_bits<3>(dmode, a, s);
        case 4: return hist_bits<4>(dmode, a, s);
        case 5: return hist_bits<5>(dmode, a, s);
        case 6: return hist_bits<6>(dmode, a, s);
        case 7: return hist_bits<7>(dmode, a, s);
        case 8: return hist_bits<8>(dmode, a, s);
        case 9: return hist_bits<9>(dmode, a, s);
        case 10: return hist_bits<10>(dmode, a, s);
        case 11: return hist_bits<11>(dmode, a, s);
        case 12: return hist_bits<12>(dmode, a, s);
        case 13: return hist_bits<13>(dmode, a, s);
        default: return hipErrorInvalidValue;
    }
}

bool scatter_available(int bits, int pairs, int rank_algo, int dmode, int geom) {
    if (geom < 0 || geom >= kGeomCount) return false;
    return scatter_kernel(bits, pairs, rank_algo, dmode, geom, 1) != nullptr;
}

hipError_t launch_scatter(int bits, int pairs, int rank_algo, int dmode, int geom, int aligned16,
                          const ScatterArgs &a, hipStream_t s) {
    if (geom < 0 || geom >= kGeomCount) return hipErrorInvalidValue;
    void *fn = scatter_kernel(bits, pairs, rank_algo, dmode, geom, aligned16);
    if (!fn) return hipErrorInvalidValue;
    // k = 3, 4 keys of up to 2^26 (the size measured): default-policy stores. A pass writes 256 MiB
    // there, as much as the Infinity Cache holds (the two ping-pong buffers, 512 MiB, do NOT fit
    // together), so part of what the next pass reads is still on die (dev/scatter_lab LAB_K4,
    // 2^26 keys: 0.105 ms per pass against 0.113 with non-temporal stores; 2^30: 1.81 vs 1.75)
    if (a.n <= ((uint64_t)1 << 26) && !pairs && dmode == kDigitShift && geom == kGeomSmall &&
        rank_algo == kRankAtomic && aligned16 && (bits == 3 || bits == 4)) {
        constexpr int TH = kGeomShape[kGeomSmall].threads, KP = kGeomShape[kGeomSmall].kpt;
        fn = bits == 3 ? reg_lines<3, TH, KP, kLineKeys, false, kDigitShift, 1>()
                       : reg_lines<4, TH, KP, kLineKeys, false, kDigitShift, 1>();
    }
    // partitions into <= 4 buckets: the line kernel's few-bucket ranking instance (CL = 2)
    if (dmode == kDigitSplit && a.nsplit < 4u) {
        constexpr int ST = kGeomShape[kGeomSmall].threads, SK = kGeomShape[kGeomSmall].kpt;
        constexpr int KT = kGeomShape[kGeomK4].threads, KK = kGeomShape[kGeomK4].kpt;
        if (fn == reinterpret_cast<void *>(&rs_scatter_lines<2, ST, SK, kLineKeys, false, kDigitSplit, 3>))
            fn = reg_lines<2, ST, SK, kLineKeys, false, kDigitSplit, 3, 2>();
        else if (fn == reinterpret_cast<void *>(&rs_scatter_lines<3, ST, SK, kLineKeys, false, kDigitSplit, 3>))
            fn = reg_lines<3, ST, SK, kLineKeys, false, kDigitSplit, 3, 2>();
        else if (fn == reinterpret_cast<void *>(&rs_scatter_lines<2, ST, SK, kLineKeysPairs, true, kDigitSplit, 2>))
            fn = reg_lines<2, ST, SK, kLineKeysPairs, true, kDigitSplit, 2, 2>();
        else if (fn == reinterpret_cast<void *>(&rs_scatter_lines<3, ST, SK, kLineKeysPairs, true, kDigitSplit, 2>))
            fn = reg_lines<3, ST, SK, kLineKeysPairs, true, kDigitSplit, 2, 2>();
        else if (fn == reinterpret_cast<void *>(&rs_scatter_lines<3, KT, KK, kLineKeys, false, kDigitSplit, 3>))
            fn = reg_lines<3, KT, KK, kLineKeys, false, kDigitSplit, 3, 2>();
    }
    // clustered-input variants of the k = 8 line kernels (rank_add_hot): both kernels are launched,
    // the device-side flag *cl_select picks the one that works (the other leaves at once: ~3 us)
    void *cl = nullptr;
    if (a.cl_select != nullptr) {
        constexpr int PT = kGeomShape[kGeomLinesPairs].threads, PK = kGeomShape[kGeomLinesPairs].kpt;
        if (fn == reinterpret_cast<void *>(&rs_scatter_lines<8, 1024, 16, kLineKeys, false, kDigitShift, 3>))
            cl = reg_lines<8, 1024, 16, kLineKeys, false, kDigitShift, 3, 1>();
        else if (fn == reinterpret_cast<void *>(&rs_scatter_lines<8, PT, PK, kLineKeysPairs, true, kDigitShift, 2>))
            cl = reg_lines<8, PT, PK, kLineKeysPairs, true, kDigitShift, 2, 1>();

    }
    // digit-group chunks, next-digit counts and raw tables exist only in the whole-line kernels: any
    // other kernel would read the unscanned counts (or the group bounds) as offsets -- refuse, never
    // sort wrongly
    const bool lines = is_line_kernel(fn);
    if ((a.raw_table || a.next_table != nullptr || a.bounds != nullptr) && !lines) return hipErrorInvalidValue;
    ScatterArgs copy = a;
    if (cl == nullptr) copy.cl_select = nullptr;  // no clustered variant: the plain kernel does the pass
    if (lines) {
        // whole-line kernels write cache lines: positions count from kout's 128-B-aligned base, the
        // slots before kout are masked like any chunk's leading slots (values: the same shift; the
        // caller checked (vout - kout) % 16 == 0, so vout's base stays 16-B aligned)
        const uintptr_t ko = (uintptr_t)a.kout, sh = ko & 127u;
        copy.kout = reinterpret_cast<uint32_t *>(ko - sh);
        if (pairs) copy.vout = reinterpret_cast<uint32_t *>((uintptr_t)a.vout - sh);
        copy.pos_shift = (uint32_t)(sh / 4u);
    }
    note_used(fn);
    if (cl != nullptr) note_used(cl);
    void *args[] = {&copy};
    hipError_t e = hipLaunchKernel(fn, dim3(a.num_chunks), dim3(kGeomShape[geom].threads), args, 0, s);
    if (e != hipSuccess || cl == nullptr) return e;
    return hipLaunchKernel(cl, dim3(a.num_chunks), dim3(kGeomShape[geom].threads), args, 0, s);
}

int scatter_blocks_per_cu(int bits, int pairs, int rank_algo, int geom, int dmode) {
    if (geom < 0 || geom >= kGeomCount) return 0;
    void *fn = scatter_kernel(bits, pairs, rank_algo, dmode, geom, 1);
    if (!fn) return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kGeomShape[geom].threads, 0) != hipSuccess)
        return 0;
    return nb;
}


hipError_t launch_histogram_joint(const HistArgs &a, hipStream_t s) {
    // one 1024-thread workgroup per chunk (the joint table fills the LDS: one per CU)
    if (a.num_chunks != kJointBins || a.split != 1 || !a.joint) return hipErrorInvalidValue;
    rs_histogram<kJointBits, 1024, kDigitShift, 1, 8, true><<<a.num_chunks, 1024, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_joint_bounds(const uint32_t *joint, const uint32_t *enable, uint32_t *bounds,
                               uint32_t *plan, uint32_t *pcounts, uint64_t n, uint64_t max_keys,
                               uint32_t snap, uint32_t weighted, hipStream_t s, const uint32_t *ctab,
                               uint32_t *rows_cnt, const uint32_t *rowone) {
    rs_joint_bounds<<<1, 1024, 0, s>>>(joint, enable, bounds, plan, pcounts, n, max_keys, snap, weighted, ctab,
                                       rows_cnt, rowone);
    return hipGetLastError();
}

hipError_t launch_scan(const ScanArgs &a, hipStream_t s) {
    rs_scan_reduce<<<a.nblocks, kScanThreads, 0, s>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    rs_scan_down<<<a.nblocks, kScanThreads, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_gather_starts(const uint32_t *table, uint32_t num_chunks, uint32_t bins,
                                uint64_t n, uint32_t *starts, hipStream_t s) {
    rs_gather_starts<<<(bins + 1 + 255) / 256, 256, 0, s>>>(table, num_chunks, bins, n, starts);
    return hipGetLastError();
}

hipError_t launch_diff_starts(const uint32_t *starts, uint32_t bins, uint32_t *hist,
                              hipStream_t s) {
    rs_diff_starts<<<(bins + 255) / 256, 256, 0, s>>>(starts, bins, hist);
    return hipGetLastError();
}

static unsigned gen_grid(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 65536 ? (g ? g : 1) : 65536);
}

hipError_t launch_top_hist_sampled(const uint32_t *keys, uint64_t n, uint32_t top_bits, uint32_t stride,
                                   uint32_t *hist, hipStream_t s) {
    const uint64_t blocks = ((n + 255) / 256 + stride - 1) / stride;  // sampled blocks
    const unsigned grid = (unsigned)std::min<uint64_t>(std::max<uint64_t>(blocks / 16, 1), 256);
    rs_top_hist_sampled<<<grid, 1024, 0, s>>>(keys, n, top_bits, stride, hist);
    return hipGetLastError();
}

hipError_t launch_sample(const uint32_t *keys, uint64_t n, uint64_t stride, uint64_t count, uint64_t row_len,
                         uint32_t *out, hipStream_t s) {
    if (row_len == 0) return hipSuccess;
    rs_sample<<<(unsigned)std::min<uint64_t>((row_len + 255) / 256, 4096), 256, 0, s>>>(keys, n, stride, count,
                                                                                        row_len, out);
    return hipGetLastError();
}

hipError_t launch_fingerprint(const uint32_t *keys, const uint32_t *vals, uint64_t n, unsigned long long *out,
                              hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, 16, s);
    if (e != hipSuccess || n == 0) return e;
    rs_fingerprint<<<(unsigned)std::min<uint64_t>((n + 255) / 256, 8192), 256, 0, s>>>(keys, vals, n, out);
    return hipGetLastError();
}

hipError_t launch_gen_uniform(uint32_t *out, uint64_t n, uint64_t seed, hipStream_t s) {
    rs_gen_uniform<<<gen_grid(n), 256, 0, s>>>(out, n, seed);
    return hipGetLastError();
}

hipError_t launch_gen_zipf(uint32_t *out, uint64_t n, uint64_t seed, const uint32_t *cdf,
                           uint64_t ranks, hipStream_t s) {
    rs_gen_zipf<<<gen_grid(n), 256, 0, s>>>(out, n, seed, cdf, ranks);
    return hipGetLastError();
}

hipError_t launch_widen(const uint32_t *in, unsigned long long *out, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    rs_widen<<<(n + 255) / 256, 256, 0, s>>>(in, out, n);
    return hipGetLastError();
}

hipError_t launch_gen_iota(uint32_t *out, uint64_t n, uint32_t base, hipStream_t s) {
    rs_gen_iota<<<gen_grid(n), 256, 0, s>>>(out, n, base);
    return hipGetLastError();
}

}  // namespace rsort
