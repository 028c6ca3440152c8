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
// Local rank (the "block-local 1-bit split sort" of the north star), two interchangeable
// algorithms giving the same unique stable order:
//   RANK_MATCH  per key: k wave64 ballots build the mask of lanes holding the same digit;
//               rank-in-wave = popcount(mask & lanes-below) + a per-wave LDS digit counter
//               bumped by ONE lane with a returning ds_add (no serial dependence between
//               slots); then a block scan of the W x R counters gives every key's tile rank.
//   RANK_SPLIT  k successive stable 1-bit splits (the reference's P5:79-159 / P7:79-191
//               algorithm), each a ballot/popcount block scan + one LDS permutation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rsort_internal.hpp"

namespace rsort {

enum RankAlgo : int { kRankMatch = 0, kRankSplit = 1 };

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, kWave);
        if (l >= (uint32_t)o) x += y;
    }
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

template <int BITS, int DMODE>
struct Digit {
    uint32_t shift;
    uint32_t nsplit;
    const uint32_t *split;
    __device__ __forceinline__ uint32_t operator()(uint32_t key) const {
        if constexpr (DMODE == kDigitShift) {
            return (key >> shift) & ((1u << BITS) - 1u);
        } else {
            uint32_t d = 0;
#pragma unroll
            for (int i = 0; i < kMaxSplitters; ++i) d += ((uint32_t)i < nsplit && key >= split[i]) ? 1u : 0u;
            return d;
        }
    }
};

// ------------------------------------------------------------------------------ histogram
// Reference: histogramKernel (Parallel7.cu:318-343) + transpose (P7:361-392, :596).
template <int BITS, int THREADS, int DMODE>
__global__ __launch_bounds__(THREADS) void rs_histogram(HistArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int HW = (R * W <= 2048) ? W : 1;  // per-wave private copies when they fit cheaply
    __shared__ uint32_t s_h[HW * R];

    const uint32_t t = threadIdx.x;
    const uint32_t c = blockIdx.x;
    for (uint32_t i = t; i < HW * R; i += THREADS) s_h[i] = 0;
    __syncthreads();

    uint32_t *my = s_h + (HW > 1 ? (t / kWave) * R : 0);
    const Digit<BITS, DMODE> dig{a.shift, a.nsplit, a.splitters};
    const uint64_t beg = (uint64_t)c * a.chunk_keys;
    const uint64_t end = min(beg + a.chunk_keys, a.n);
    uint64_t tail = beg;
    if (a.vec) {
        const uint4 *p = reinterpret_cast<const uint4 *>(a.keys + beg);
        const uint32_t nvec = (uint32_t)((end - beg) / 4);
        constexpr int U = 4;
        for (uint32_t v0 = t; v0 < nvec; v0 += THREADS * U) {
            uint4 q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t v = v0 + u * THREADS;
                q[u] = v < nvec ? p[v] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (v0 + u * THREADS < nvec) {
                    atomicAdd(&my[dig(q[u].x)], 1u);
                    atomicAdd(&my[dig(q[u].y)], 1u);
                    atomicAdd(&my[dig(q[u].z)], 1u);
                    atomicAdd(&my[dig(q[u].w)], 1u);
                }
            }
        }
        tail = beg + (uint64_t)nvec * 4;
    }
    for (uint64_t i = tail + t; i < end; i += THREADS) atomicAdd(&my[dig(a.keys[i])], 1u);
    __syncthreads();
    for (uint32_t d = t; d < R; d += THREADS) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < HW; ++w) s += s_h[w * R + d];
        a.table[(uint64_t)d * a.num_chunks + c] = s;
    }
}

// ------------------------------------------------------------------------------ table scan
// Exclusive scan of the column-major chunk x digit table, == the column-major scan of
// Baseline4.cu:127-138 / P7's transpose-scan-transpose. Two launches: segment sums, then
// each segment adds the sum of the segments before it (<= a few thousand values, read from
// L2) and scans itself.
__global__ __launch_bounds__(kScanThreads) void rs_scan_reduce(ScanArgs a) {
    __shared__ uint32_t s_ws[kScanThreads / kWave];
    const uint64_t base = (uint64_t)blockIdx.x * kScanSegment + (uint64_t)threadIdx.x * kScanPerThread;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) s += (base + i < a.m) ? a.table[base + i] : 0u;
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

// ------------------------------------------------------------------------------ scatter
// Reference: sortLocallyDataBlocks (P7:193-251: scanLocallyBlocksUnroll2Kernel :79-141 +
// scatterLocallyBlocksKernel :143-191, or the in-SMEM P5:79-159) fused with scatterKernel
// (P7:253-304). Per tile: load (coalesced, wave-striped: lane l of wave w holds tile
// positions w*64*KPT + j*64 + l), rank locally, stage the tile in LDS in digit order, then
// write each digit's run to global at table[digit][chunk] + (earlier tiles' count) +
// (position - first position of the digit in the tile) -- the firstIndices rank formula of
// P7:293-294 with the running offset kept in registers.
template <int BITS, int THREADS, int KPT, bool PAIRS, int RANK, int DMODE>
__global__ __launch_bounds__(THREADS) void rs_scatter(ScatterArgs a) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int W = THREADS / kWave;
    constexpr int SEG = kWave * KPT;            // tile positions per wave
    constexpr uint32_t T = THREADS * KPT;       // tile keys
    constexpr int DPT = (R > THREADS) ? (int)(R / THREADS) : 1;  // digits owned per thread
    constexpr uint32_t NCNT = (RANK == kRankMatch) ? W * R : R;

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
    for (uint64_t tb = cbeg; tb < cend; tb += T) {
        const uint32_t valid = (uint32_t)min<uint64_t>((uint64_t)T, cend - tb);
        uint32_t key[KPT];
        uint32_t val[PAIRS ? KPT : 1];
        uint32_t dg[KPT];
        // ---- load (positions past the end become digit R-1, which sorts them last)
        if (valid == T) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                key[j] = a.kin[tb + base + j * kWave];
                if constexpr (PAIRS) val[j] = a.vin[tb + base + j * kWave];
            }
#pragma unroll
            for (int j = 0; j < KPT; ++j) dg[j] = dig(key[j]);
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t p = base + j * kWave;
                key[j] = p < valid ? a.kin[tb + p] : 0xFFFFFFFFu;
                if constexpr (PAIRS) val[j] = p < valid ? a.vin[tb + p] : 0u;
                dg[j] = p < valid ? dig(key[j]) : R - 1;
            }
        }
        for (uint32_t i = t; i < NCNT; i += THREADS) s_cnt[i] = 0;
        __syncthreads();

        uint32_t rk[KPT];
        if constexpr (RANK == kRankMatch) {
            // ---- wave peer-match ranking; counters s_cnt[w][digit]
            const uint64_t below = lanes_below();
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                uint64_t m = ~0ull;
#pragma unroll
                for (int b = 0; b < BITS; ++b) {
                    const uint32_t bit = (dg[j] >> b) & 1u;
                    const uint64_t bal = __ballot(bit);
                    m &= bit ? bal : ~bal;
                }
                const uint32_t pre = (uint32_t)__popcll(m & below);
                uint32_t old = 0;
                if (pre == 0) old = atomicAdd(&s_cnt[w * R + dg[j]], (uint32_t)__popcll(m));
                old = __shfl(old, (int)__ffsll((unsigned long long)m) - 1, kWave);
                rk[j] = old + pre;
            }
            __syncthreads();
            // ---- digit scan: per owned digit, exclusive over waves; block scan over digits
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
            // ---- stage the tile in digit order
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t pos = s_cnt[w * R + dg[j]] + rk[j];
                s_keys[pos] = key[j];
                if constexpr (PAIRS) s_vals[pos] = val[j];
            }
            __syncthreads();
            // ---- write each digit's run: consecutive threads -> consecutive addresses
            if (a.local_only) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t i = t + j * THREADS;
                    if (i < valid) {
                        a.kout[tb + i] = s_keys[i];
                        if constexpr (PAIRS) a.vout[tb + i] = s_vals[i];
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t i = t + j * THREADS;
                    if (i < valid) {
                        const uint32_t k = s_keys[i];
                        const uint32_t pos = s_delta[dig(k)] + i;
                        a.kout[pos] = k;
                        if constexpr (PAIRS) a.vout[pos] = s_vals[i];
                    }
                }
            }
        } else {
            // ---- RANK_SPLIT: k stable 1-bit splits in LDS (reference P5:89-146 / P7:79-191)
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
        }
    }
}

// ------------------------------------------------------------------------------ small kernels
// starts[d] = scanned table[d][0] (global start of digit d), starts[bins] = n.
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
template <int BITS>
static hipError_t hist_bits(int dmode, const HistArgs &a, hipStream_t s) {
    if (dmode == kDigitSplit) {
        if constexpr (BITS <= 4) {
            rs_histogram<BITS, kThreads, kDigitSplit><<<a.num_chunks, kThreads, 0, s>>>(a);
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
    rs_histogram<BITS, kThreads, kDigitShift><<<a.num_chunks, kThreads, 0, s>>>(a);
    return hipGetLastError();
}

template <int BITS, bool PAIRS, int RANK, int DMODE>
static void *scatter_fn() {
    return reinterpret_cast<void *>(&rs_scatter<BITS, kThreads, kKeysPerThread, PAIRS, RANK, DMODE>);
}

template <int BITS>
static void *scatter_pick(int pairs, int rank, int dmode) {
    if (dmode == kDigitSplit) {
        if constexpr (BITS <= 4) {
            return pairs ? scatter_fn<BITS, true, kRankMatch, kDigitSplit>()
                         : scatter_fn<BITS, false, kRankMatch, kDigitSplit>();
        }
        return nullptr;
    }
    if (rank == kRankSplit)
        return pairs ? scatter_fn<BITS, true, kRankSplit, kDigitShift>()
                     : scatter_fn<BITS, false, kRankSplit, kDigitShift>();
    return pairs ? scatter_fn<BITS, true, kRankMatch, kDigitShift>()
                 : scatter_fn<BITS, false, kRankMatch, kDigitShift>();
}

static void *scatter_kernel(int bits, int pairs, int rank, int dmode) {
    switch (bits) {
        case 1: return scatter_pick<1>(pairs, rank, dmode);
        case 2: return scatter_pick<2>(pairs, rank, dmode);
        case 3: return scatter_pick<3>(pairs, rank, dmode);
        case 4: return scatter_pick<4>(pairs, rank, dmode);
        case 5: return scatter_pick<5>(pairs, rank, dmode);
        case 6: return scatter_pick<6>(pairs, rank, dmode);
        case 7: return scatter_pick<7>(pairs, rank, dmode);
        case 8: return scatter_pick<8>(pairs, rank, dmode);
        case 9: return scatter_pick<9>(pairs, rank, dmode);
        case 10: return scatter_pick<10>(pairs, rank, dmode);
        case 11: return scatter_pick<11>(pairs, rank, dmode);
        case 12: return scatter_pick<12>(pairs, rank, dmode);
        default: return nullptr;
    }
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
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scatter(int bits, int pairs, int rank_algo, int dmode, const ScatterArgs &a,
                          hipStream_t s) {
    void *fn = scatter_kernel(bits, pairs, rank_algo, dmode);
    if (!fn) return hipErrorInvalidValue;
    ScatterArgs copy = a;
    void *args[] = {&copy};
    return hipLaunchKernel(fn, dim3(a.num_chunks), dim3(kThreads), args, 0, s);
}

int scatter_blocks_per_cu(int bits, int pairs, int rank_algo) {
    void *fn = scatter_kernel(bits, pairs, rank_algo, kDigitShift);
    if (!fn) return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kThreads, 0) != hipSuccess) return 0;
    return nb;
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

hipError_t launch_gen_uniform(uint32_t *out, uint64_t n, uint64_t seed, hipStream_t s) {
    rs_gen_uniform<<<gen_grid(n), 256, 0, s>>>(out, n, seed);
    return hipGetLastError();
}

hipError_t launch_gen_zipf(uint32_t *out, uint64_t n, uint64_t seed, const uint32_t *cdf,
                           uint64_t ranks, hipStream_t s) {
    rs_gen_zipf<<<gen_grid(n), 256, 0, s>>>(out, n, seed, cdf, ranks);
    return hipGetLastError();
}

hipError_t launch_gen_iota(uint32_t *out, uint64_t n, uint32_t base, hipStream_t s) {
    rs_gen_iota<<<gen_grid(n), 256, 0, s>>>(out, n, base);
    return hipGetLastError();
}

}  // namespace rsort
