// dev/pairs_variants.hpp -- the round-3..5 lab variants of rs_scatter_pairs (the C4 pass), kept out of the
// library: rs_scatter_pairs_lab<BITS, THREADS, KPT, CL, PF, OPT> is the kernel as it was
// at the end of round 5 with its measurement knobs (PF = 2 tiles of loads in flight; OPT bits below). With
// PF = 1, OPT = 0 it is the library's rs_scatter_pairs. Included by dev/pairs_lab.hip after the library's
// kernels (it uses their helpers); every knob's measurement is in dev/LOG.md.
#pragma once
namespace rsort {
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
// rs_scatter_lines.
// (lab knobs, dev/pairs_lab.hip: PF = 2 tiles of loads in flight; OPT & 1 non-temporal loads, OPT & 2
// the next tile's loads issued before the rank loop instead of after it, OPT & 4 keys and values
// staged interleaved, OPT & 8 step 4 deferred to after the next tile's rank phase,
// OPT & 16 / 32 the next tile's loads issued after step 2 / step 3 instead of after the rank phase,
// OPT & 64 keys and values through ONE staging array in turn: steps 3 and 4 for the keys, then for the
// values at the same slots (kept in registers) -- half the LDS, so two workgroups fit per CU)
template <int BITS, int THREADS, int KPT, int CL = 0, int PF = 1, int OPT = 0>
__global__ __launch_bounds__(THREADS, ((OPT & 64) && THREADS <= 512) ? 4 : 1) void rs_scatter_pairs_lab(ScatterArgs a) {
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
    // OPT & 4: one interleaved {key, value} array (8-B stores per pair) instead of two
    constexpr bool IL = (OPT & 4) != 0;
    constexpr bool DEFER = (OPT & 8) != 0;
    constexpr bool SQ = (OPT & 64) != 0;
    static_assert(!(SQ && (IL || DEFER)), "sequential staging: two plain arrays' worth of work in one");
    __shared__ __attribute__((aligned(16))) uint32_t s_k[IL ? 4 : CAP + 36];
    __shared__ __attribute__((aligned(16))) uint32_t s_v[(IL || SQ) ? 4 : CAP + 36];
    __shared__ __attribute__((aligned(16))) uint2 s_kv[IL ? CAP + 36 : 2];
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
                k[j] = (OPT & 1) ? __builtin_nontemporal_load(tk + j * kWave) : tk[j * kWave];
                v[j] = (OPT & 1) ? __builtin_nontemporal_load(tv + j * kWave) : tv[j * kWave];
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
        u32x4 kv, vv;
        if constexpr (IL) {
            const u32x4 p01 = *reinterpret_cast<const u32x4 *>(&s_kv[li]);
            const u32x4 p23 = *reinterpret_cast<const u32x4 *>(&s_kv[li + 2]);
            kv = u32x4{p01.x, p01.z, p23.x, p23.z};
            vv = u32x4{p01.y, p01.w, p23.y, p23.w};
        } else {
            kv = *reinterpret_cast<const u32x4 *>(&s_k[li]);
            vv = *reinterpret_cast<const u32x4 *>(&s_v[li]);
        }
        const uint64_t gp = (uint64_t)(lr.x + q);
        const uint32_t lo = lr.y >> 16;
        if (lo <= q) {
            __builtin_nontemporal_store(kv, reinterpret_cast<u32x4 *>(a.kout + gp));
            __builtin_nontemporal_store(vv, reinterpret_cast<u32x4 *>(a.vout + gp));
        } else {
            // the chunk's first line of this digit: lanes below lo belong to the previous chunk
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x)
                if (lo <= q + x) {
                    a.kout[gp + x] = kv[x];
                    a.vout[gp + x] = vv[x];
                }
        }
    };

    // SQ: one array's quad of whole line item / QPL from the staging array (the keys' or the values')
    auto store_one = [&](uint32_t item, uint32_t *__restrict__ dst) {
        const uint32_t V = item / QPL, q = (item % QPL) * 4u;
        const uint2 lr = s_lrec[V];
        const u32x4 kv = *reinterpret_cast<const u32x4 *>(&s_k[(lr.y & 0xFFFFu) + q]);
        const uint64_t gp = (uint64_t)(lr.x + q);
        const uint32_t lo = lr.y >> 16;
        if (lo <= q) {
            __builtin_nontemporal_store(kv, reinterpret_cast<u32x4 *>(dst + gp));
        } else {
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x)
                if (lo <= q + x) dst[gp + x] = kv[x];
        }
    };
    // SQ: one array's tails (from the staging array) into its carry registers, and its whole lines out
    auto output_one = [&](const uint32_t S, const uint32_t wl, const uint32_t pending, const uint32_t nlines,
                          uint32_t (&cr)[CPT], uint32_t *__restrict__ dst) {
        const uint32_t tl0 = S + wl * G + sub * CPT;
        const uint32_t ncarry = pending - wl * G;
#pragma unroll
        for (uint32_t i = 0; i < CPT; i += 4) {
            if (sub * CPT + i >= ncarry) break;
            const u32x4 q4 = *reinterpret_cast<const u32x4 *>(&s_k[tl0 + i]);
            cr[i] = q4.x; cr[i + 1] = q4.y; cr[i + 2] = q4.z; cr[i + 3] = q4.w;
        }
        const uint32_t nq = nlines * QPL;
        for (uint32_t item = t; item < nq; item += 2 * THREADS) {
            store_one(item, dst);
            if (item + THREADS < nq) store_one(item + THREADS, dst);
        }
    };

    RS_STAMP_DECL
    // ---- 4. (of a tile) the tails back into the carry registers (the quads holding any); whole lines
    //      out. DEFER: run after the NEXT tile's rank phase instead of at the end of the tile.
    auto output = [&](const uint32_t S, const uint32_t wl, const uint32_t pending, const uint32_t nlines,
                      const uint32_t cnt) {
        {
            const uint32_t tl0 = S + wl * G + sub * CPT;  // quad-aligned
            const uint32_t ncarry = pending - wl * G;
#pragma unroll
            for (uint32_t i = 0; i < CPT; i += 4) {
                if (sub * CPT + i >= ncarry) break;
                u32x4 kq, vq;
                if constexpr (IL) {
                    const u32x4 p01 = *reinterpret_cast<const u32x4 *>(&s_kv[tl0 + i]);
                    const u32x4 p23 = *reinterpret_cast<const u32x4 *>(&s_kv[tl0 + i + 2]);
                    kq = u32x4{p01.x, p01.z, p23.x, p23.z};
                    vq = u32x4{p01.y, p01.w, p23.y, p23.w};
                } else {
                    kq = *reinterpret_cast<const u32x4 *>(&s_k[tl0 + i]);
                    vq = *reinterpret_cast<const u32x4 *>(&s_v[tl0 + i]);
                }
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
    uint32_t pS = 0, pwl = 0, ppend = 0, pnl = 0, pcnt = 0;  // DEFER: the staged tile's step-4 state
    bool have_prev = false;

    // The tile step. PF = 1: the next tile's loads go into nkey at the end of the rank phase and
    // move into key at the end of the step. PF = 2: two register sets alternate (the loop is unrolled
    // by two); a tile's set takes the loads of the tile two ahead as soon as it is staged.
    uint32_t hotd = 0xFFFFFFFFu;
    auto tile_step = [&](const uint64_t tb, uint32_t (&key)[KPT], uint32_t (&val)[KPT]) {
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
            uint32_t nkey[PF == 1 ? KPT : 1], nval[PF == 1 ? KPT : 1];
            if constexpr (PF == 1 && (OPT & 2)) {
                if (nb < cend) load_tile(nb, nkey, nval);
            }
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
                        const uint32_t r = hot_rank(o[u], dig(key[j]), cc[u], mm[u]);
                        rk[j / 2] = (j & 1) ? (rk[j / 2] | (r << 16)) : r;
                    }
                }
            } else if (full) {
    #pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t dj = dig(key[j]);
                    const uint32_t r = CL ? rank_add_hot(&s_cnt[w * RS], dj, hotd) : rank_add(&s_cnt[w * RS], dj);
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
            if constexpr (PF == 1 && !(OPT & (2 | 16 | 32))) {
                if (nb < cend) load_tile(nb, nkey, nval);
            }
            if constexpr (DEFER) {
                // the previous tile's output: its stores then have steps 2-3 of this tile to drain
                // before the next vmcnt wait (at the next rank phase), instead of none
                if (have_prev) output(pS, pwl, ppend, pnl, pcnt);
                have_prev = true;
            }
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
                    if constexpr (IL) {
                        *reinterpret_cast<u32x4 *>(&s_kv[S + sub * CPT + i]) = u32x4{ck[i], cv[i], ck[i + 1], cv[i + 1]};
                        *reinterpret_cast<u32x4 *>(&s_kv[S + sub * CPT + i + 2]) =
                            u32x4{ck[i + 2], cv[i + 2], ck[i + 3], cv[i + 3]};
                    } else {
                        *reinterpret_cast<u32x4 *>(&s_k[S + sub * CPT + i]) = u32x4{ck[i], ck[i + 1], ck[i + 2], ck[i + 3]};
                        if constexpr (!SQ)
                            *reinterpret_cast<u32x4 *>(&s_v[S + sub * CPT + i]) = u32x4{cv[i], cv[i + 1], cv[i + 2], cv[i + 3]};
                    }
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
            if constexpr (PF == 1 && (OPT & 16)) {
                if (nb < cend) load_tile(nb, nkey, nval);
            }

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
            uint32_t sidx[SQ ? KPT : 1];  // SQ: every slot's staging index, for the values after the keys
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
                    if constexpr (IL) {
                        s_kv[idx] = make_uint2(key[j], val[j]);
                    } else if constexpr (SQ) {
                        s_k[idx] = key[j];
                        sidx[j] = idx;
                    } else {
                        s_k[idx] = key[j];
                        s_v[idx] = val[j];
                    }
                }
            }
            // PF = 2: this tile's registers are free (staged): the tile after next goes into them, in
            // flight through this tile's output and the whole next tile
            if constexpr (PF == 2) {
                if (nb + T < cend) load_tile(nb + T, key, val);
            }
            __syncthreads();
            RS_STAMP(3);
            if constexpr (PF == 1 && (OPT & 32)) {
                if (nb < cend) load_tile(nb, nkey, nval);
            }

            if constexpr (SQ) {
                // the keys' lines and tails; then the values through the same slots: their carry into the
                // segment heads, staged at the keys' indices, their lines and tails
                output_one(S, wl, pending, nlines, ck, a.kout);
                __syncthreads();
                // (dword by dword: no barrier separates these from the staging below, so a whole quad
                // past the carry's end could land after a staged value)
    #pragma unroll
                for (uint32_t i = 0; i < CPT; ++i)
                    if (sub * CPT + i < carry) s_k[S + sub * CPT + i] = cv[i];
    #pragma unroll
                for (int j = 0; j < KPT; ++j) s_k[sidx[j]] = val[j];
                __syncthreads();
                output_one(S, wl, pending, nlines, cv, a.vout);
                if (wl > 0) inv = 0;
                carry = pending - wl * G;
                g_run += cnt;
            } else if constexpr (DEFER) {
                pS = S;
                pwl = wl;
                ppend = pending;
                pnl = nlines;
                pcnt = cnt;
            } else {
                output(S, wl, pending, nlines, cnt);
            }
            if constexpr (PF == 1) {
    #pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    key[j] = nkey[j];
                    val[j] = nval[j];
                }
            }
    };
    uint32_t keyA[KPT], valA[KPT];
    if (cbeg < cend) load_tile(cbeg, keyA, valA);
    if constexpr (PF == 1) {
        for (uint64_t tb = cbeg; tb < cend; tb += T) tile_step(tb, keyA, valA);
    } else {
        uint32_t keyB[KPT], valB[KPT];
        if (cbeg + T < cend) load_tile(cbeg + T, keyB, valB);
        for (uint64_t tb = cbeg; tb < cend; tb += 2 * T) {
            tile_step(tb, keyA, valA);
            if (tb + T < cend) tile_step(tb + T, keyB, valB);
        }
    }
    if constexpr (DEFER) {
        if (have_prev) output(pS, pwl, ppend, pnl, pcnt);
    }
    // ---- chunk end: the carries (slots inv .. carry - 1 from the line at g_run - carry)
    if (cbeg < cend) {
        const uint64_t A = (uint64_t)(g_run - carry);
#pragma unroll
        for (uint32_t i = 0; i < CPT; ++i) {
            const uint32_t x = sub * CPT + i;
            if (x >= inv && x < carry) {
                a.kout[A + x] = ck[i];
                a.vout[A + x] = cv[i];
            }
        }
    }
    RS_STAMP_FLUSH();
}
}  // namespace rsort
