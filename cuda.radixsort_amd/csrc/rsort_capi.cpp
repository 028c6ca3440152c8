// rsort_capi.cpp -- host driver + C ABI (include/rsort.h) of the gfx950 LSD radix sort.
//
// Replaces the reference's per-digit driver sortByDevice (Parallel7.cu:530-639) and the
// dispatcher's device branch (Parallel7.cu:641-662). Differences by design:
//   * workspace is planned once (rsort_plan) and passed in, not cudaMalloc'ed per call or
//     kept in function statics (P7:203-218, :489-505); the host entry caches one per device;
//   * one stream, no host synchronisation inside the pass loop (P7 syncs after every launch
//     and round-trips the block sums through the host every pass, P7:224-235, :514-519);
//   * errors are returned as rsort_status, never exit() (common.h:6-16).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "rsort.h"
#include "rsort_internal.hpp"

using namespace rsort;

namespace {

constexpr int kVersion = 100;  // 0.1.0
std::atomic<int> g_rank_algo{RSORT_RANK_MATCH};
std::atomic<int> g_group_chunks{1};
std::atomic<int> g_table_fault{0};  // rsort_inject_table_fault (tests)
std::atomic<int> g_rank_fault{0};   // rsort_inject_rank_fault (tests)

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// ------------------------------------------------------------------------------ profiler
struct ProfRec {
    int phase;
    int64_t keys;
    hipEvent_t a, b;
};

struct Profiler {
    std::mutex mu;
    bool on = false;
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> pool;

    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
};
Profiler g_prof;
thread_local int t_prof_paused = 0;  // profile_pause

// RAII scope: records a start event now and a stop event on destruction (same stream).
struct PhaseScope {
    bool active = false;
    ProfRec rec{};
    hipStream_t s;
    PhaseScope(int phase, int64_t keys, hipStream_t stream) : s(stream) {
        if (t_prof_paused > 0) return;
        std::lock_guard<std::mutex> g(g_prof.mu);
        if (!g_prof.on) return;
        rec.phase = phase;
        rec.keys = keys;
        rec.a = g_prof.get();
        rec.b = g_prof.get();
        if (!rec.a || !rec.b) return;
        if (hipEventRecord(rec.a, s) != hipSuccess) return;
        active = true;
    }
    ~PhaseScope() {
        if (!active) return;
        std::lock_guard<std::mutex> g(g_prof.mu);
        if (hipEventRecord(rec.b, s) == hipSuccess) g_prof.recs.push_back(rec);
    }
};

int hip_status(hipError_t e) { return e == hipSuccess ? RSORT_OK : RSORT_ERR_HIP; }

bool aligned4(const void *p) { return ((uintptr_t)p & 3u) == 0; }

// The whole-line scatter kernels can write these outputs: any 4-B-aligned kout (launch_scatter
// counts positions from its 128-B-aligned base, i.e. every position moves up by the < 32 keys
// between that base and kout -- so n plus that shift must still fit the kernels' 32-bit positions);
// values at a multiple of 16 B from the keys.
bool line_capable(const void *kout, const void *vout, int pairs, int64_t n) {
    if (!aligned4(kout)) return false;
    if (n + (int64_t)(((uintptr_t)kout & 127u) / 4u) >= ((int64_t)1 << 32)) return false;
    return !pairs || ((((uintptr_t)vout - (uintptr_t)kout) & 15u) == 0);
}

// ------------------------------------------------------------------------------ planning
int device_cus() {
    int dev = 0, count = 0, c = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return c;
}

// log2 of the smallest k = 4 keys-only sort on 1024-thread line tiles (default 28; RSORT_K4_LINES_LG
// under RSORT_LAB=1 for A/B runs)
int k4_lines_lg() {
    static const int v = [] {
        const char *e = lab_env("RSORT_K4_LINES_LG");
        const int x = e ? atoi(e) : 0;
        return (x >= 16 && x <= 32) ? x : 28;
    }();
    return v;
}

// Tile geometry for one sort: for k = 5..8, keys-only sorts write whole 64-B lines from
// 16384-key tiles (rs_scatter_lines), pairs from 8192-key tiles; k <= 4 keys
// use 8192-key tiles; everything else 4096-key tiles -- as do inputs too small to give every
// CU two large tiles.
int choose_geom(int64_t n, int k, int pairs, int rank, int partition, int cus) {
    const int64_t enough = 2 * (int64_t)(cus > 0 ? cus : 256);
    // partitions: 4096-key tiles (measured at 2^30 keys into 8 ranges: 1024-thread 16384-key
    // tiles need 4-bit bucket digits, i.e. 15 splitter compares per key, and were 1.3x slower)
    if (k >= 13) return kGeomXL;
    // keys-only partitions of large inputs: 8192-key tiles of 512 threads (3-bit bucket digits keep
    // a digit's thread group inside one wave; runs of ~1024 keys per bucket and tile)
    if (partition && !pairs && n >= enough * geom_tile_keys(kGeomK4)) return kGeomK4;
    if (partition || rank == RSORT_RANK_SPLIT) return kGeomSmall;
    if (k >= 5 && k <= 8 && !pairs && n >= enough * geom_tile_keys(kGeomLines)) return kGeomLines;
    // k = 4 keys from 2^28 on: the same 1024-thread line tiles (dev/scatter_lab LAB_K4 at 2^30:
    // 1.61 ms per pass against 1.75 ms with 4096-key tiles; at 2^26 0.120 against 0.113)
    if (k == 4 && !pairs && n >= ((int64_t)1 << k4_lines_lg())) return kGeomLines;
    if (k >= 5 && k <= 8 && pairs && n >= enough * geom_tile_keys(kGeomLinesPairs)) return kGeomLinesPairs;
    // k = 3, 4 keys run 4096-key tiles through rs_scatter_lines (kGeomSmall's shape; whole 128-B
    // lines: 2^26 keys, k = 4: 0.117 vs 0.144 ms per pass, dev/scatter_lab.hip); k <= 2 keeps
    // rs_scatter's 8192-key tiles
    if (k <= 2 && !pairs && n >= enough * geom_tile_keys(kGeomK4)) return kGeomK4;
    return kGeomSmall;
}

// Digit-group chunks (rs_histogram_joint, rsort_kernels.hip): k = 8 plans with exactly 2^8
// chunks of line tiles. Every second pass then reads no keys for its histogram.
bool joint_plan(const rsort_plan &p) {
    return p.k_bits == kJointBits && p.num_chunks == (int64_t)kJointBins && p.passes >= 2 &&
           (geom_from_shape(p.threads, p.tile_keys, p.pairs) == (p.pairs ? kGeomLinesPairs : kGeomLines));
}

// RSORT_CUT_WEIGHTS=0 under RSORT_LAB=1: cut plans with equal key counts per chunk (A/B runs)
bool cut_weights() {
    static const bool v = [] {
        const char *e = lab_env("RSORT_CUT_WEIGHTS");
        return !(e != nullptr && e[0] == '0');
    }();
    return v;
}

// RSORT_PIECE_ROWS=0 under RSORT_LAB=1: cut plans count all their pieces from the keys (no per-chunk
// joint-count rows; the round-4 scheme) for A/B runs
bool piece_rows() {
    static const bool v = [] {
        const char *e = lab_env("RSORT_PIECE_ROWS");
        return !(e != nullptr && e[0] == '0');
    }();
    return v;
}

// RSORT_NX_TAIL=1 under RSORT_LAB=1: next-digit plans scan each pass's table in its last workgroup
// (the round-3 scheme) instead of every workgroup of the next pass summing the raw counts (A/B runs)
bool nx_tail() {
    static const bool v = [] {
        const char *e = lab_env("RSORT_NX_TAIL");
        return e != nullptr && e[0] != '\0' && e[0] != '0';
    }();
    return v;
}

// Next-digit counts (rs_scatter_lines, k = 3, 4 keys): each pass adds the next pass's chunk table
// from where it writes every key, so only pass 0 reads keys for a histogram. Needs the line
// kernel (lane-ordered ranks, line-capable outputs: checked per sort) and a second table.
bool next_plan(const rsort_plan &p) {
    const int g = geom_from_shape(p.threads, p.tile_keys, p.pairs);
    return (p.k_bits == 3 || p.k_bits == 4) && !p.pairs && p.passes >= 2 && (g == kGeomSmall || g == kGeomLines);
}

int plan_fill(int64_t n, int k, int pairs, int64_t tpc, rsort_plan *p, int partition = 0) {
    if (!p) return RSORT_ERR_ARG;
    if (k < kMinBits || k > kMaxBits) return RSORT_ERR_BITS;
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (tpc < 0) return RSORT_ERR_ARG;
    memset(p, 0, sizeof(*p));
    const int rank = g_rank_algo.load();
    const int cus = device_cus();
    const int geom = choose_geom(n, k, pairs, rank, partition, cus);
    const int tile = geom_tile_keys(geom);
    p->n = n;
    p->k_bits = k;
    p->passes = (32 + k - 1) / k;
    p->bins = 1 << k;
    p->threads = kGeomShape[geom].threads;
    p->tile_keys = tile;
    p->pairs = pairs ? 1 : 0;
    const int64_t tiles = std::max<int64_t>(1, (n + tile - 1) / tile);
    if (tpc == 0) {
        // one resident wave of workgroups: as many chunks as the scatter kernel keeps resident
        // (of the kernel this plan's scatter runs: a partition's digit is a bucket)
        int bpc = cus > 0 ? scatter_blocks_per_cu(k, pairs, internal_rank(partition ? RSORT_RANK_MATCH : rank), geom,
                                                  partition ? kDigitSplit : kDigitShift) : 0;
        if (bpc <= 0) bpc = 2;
        const int64_t target = std::max<int64_t>(1, (int64_t)(cus > 0 ? cus : 256) * bpc);
        tpc = (tiles + target - 1) / target;
    }
    p->tiles_per_chunk = tpc;
    p->chunk_keys = tpc * tile;
    p->num_chunks = (tiles + tpc - 1) / tpc;
    p->table_entries = (int64_t)p->bins * p->num_chunks;
    p->scan_blocks = (p->table_entries + kScanSegment - 1) / kScanSegment;
    size_t ws = align256((size_t)n * 4);                     // ping-pong keys
    if (pairs) ws += align256((size_t)n * 4);                // ping-pong values
    ws += align256((size_t)p->table_entries * 4);            // chunk x digit table
    ws += align256((size_t)p->scan_blocks * 4);              // scan block sums
    ws += align256((size_t)(p->bins + 1) * 4);               // bucket starts (partition / top hist)
    ws += 256;                                               // check words (tail-scan counter, check word)
    if (joint_plan(*p)) {
        ws += align256((size_t)kJointBins * kJointBins * 4 + 4);  // joint counts [next digit][digit], rows counter
        ws += align256((size_t)2 * kBoundsWords * 4);             // group bounds of passes 1 and 3
        ws += align256((size_t)kPlanWords * 4);                   // cut plan
        ws += align256((size_t)kPieceSlots * kJointBins * 4);     // its piece counts
        ws += align256(((size_t)kRowsWords + kJointBins * kJointBins) * 4);  // per-chunk joint-count rows (64 MiB)
    }
    if (!partition && next_plan(*p)) {
        ws += align256((size_t)p->table_entries * 4);  // the next pass's table
        ws += align256((size_t)p->table_entries * 4);  // raw-table offsets: the third table of the rotation
    }
    p->workspace_bytes = ws;
    return RSORT_OK;
}

// Digit bits of a partition of n keys into num_buckets key ranges: enough for the buckets, and
// enough that the whole-line scatter kernel of the partition's tile shape (choose_geom) gives
// each digit at most one wave of threads.
int partition_bits(int64_t n, int num_buckets, int pairs) {
    const int geom = choose_geom(n, 0, pairs, RSORT_RANK_MATCH, 1, device_cus());
    int bits = 1;
    while ((1 << bits) < num_buckets || (kGeomShape[geom].threads >> bits) > kWave) ++bits;
    return bits;
}

struct Carve {
    uint32_t *tmp_k, *tmp_v, *table, *bsums, *starts, *joint, *bounds, *plan, *pcounts, *table2, *done, *table3;
    uint32_t *rows, *rows_cnt;  // joint plans: per-chunk joint-count rows (HistArgs::rows), their counter
};

Carve carve(const rsort_plan &p, void *ws) {
    Carve c{};
    char *q = (char *)ws;
    c.tmp_k = (uint32_t *)q;
    q += align256((size_t)p.n * 4);
    if (p.pairs) {
        c.tmp_v = (uint32_t *)q;
        q += align256((size_t)p.n * 4);
    }
    c.table = (uint32_t *)q;
    q += align256((size_t)p.table_entries * 4);
    c.bsums = (uint32_t *)q;
    q += align256((size_t)p.scan_blocks * 4);
    c.starts = (uint32_t *)q;
    q += align256((size_t)(p.bins + 1) * 4);
    c.done = (uint32_t *)q;
    q += 256;
    if (joint_plan(p)) {
        c.joint = (uint32_t *)q;
        c.rows_cnt = c.joint + kJointBins * kJointBins;  // (cleared with the joint counts)
        q += align256((size_t)kJointBins * kJointBins * 4 + 4);
        c.bounds = (uint32_t *)q;
        q += align256((size_t)2 * kBoundsWords * 4);
        c.plan = (uint32_t *)q;
        q += align256((size_t)kPlanWords * 4);
        c.pcounts = (uint32_t *)q;
        q += align256((size_t)kPieceSlots * kJointBins * 4);
        c.rows = (uint32_t *)q;
        q += align256(((size_t)kRowsWords + kJointBins * kJointBins) * 4);
    }
    if (next_plan(p)) {
        c.table2 = (uint32_t *)q;
        q += align256((size_t)p.table_entries * 4);
        c.table3 = (uint32_t *)q;
    }
    return c;
}

// ------------------------------------------------------------------------------ pass pieces
// Joint pass (pass p of a joint_plan counting for pass p + 1): one workgroup per chunk counts
// this pass's table and the joint counts; then the chunks of pass p + 1 (its digit groups, or
// the cut plan). enable: nullptr, or the previous odd pass's mode: the joint count runs after whole
// digit groups and after a cut plan (both leave the joint counts cleared: the copy-mode histogram, the
// cut plan's scan), not after fixed chunks. After a cut plan the input is clustered: the joint count
// adds runs of equal pairs once (rs_histogram's run path), so pass 3 gets its own cut plan too.
int do_histogram_joint(const rsort_plan &p, const uint32_t *keys, int shift, uint32_t *table,
                       uint32_t *joint, const uint32_t *enable, hipStream_t s, bool zero_joint,
                       uint32_t *rows, uint32_t *rows_cnt, uint32_t *done = nullptr) {
    HistArgs a{};
    a.done = done;
    a.rows = rows;
    a.rows_cnt = rows_cnt;
    a.keys = keys;
    a.table = table;
    a.n = (uint64_t)p.n;
    a.chunk_keys = (uint64_t)p.chunk_keys;
    a.num_chunks = (uint32_t)p.num_chunks;
    a.shift = (uint32_t)shift;
    a.vec = (((uintptr_t)keys & 15u) == 0) ? 1u : 0u;
    a.split = 1;
    a.joint = joint;
    a.joint_enable = enable;
    PhaseScope ps(RSORT_PHASE_HISTOGRAM, p.n, s);
    // the first joint count of a sort clears the counts; a later one finds them cleared by the
    // copy-mode histogram that used them (or, where that pass fell back, is disabled by `enable`)
    // (the rows counter sits after the joint counts: cleared with them)
    // (16 bytes past the counts, inside the 256-B-aligned region: a fill of a multiple of 16 bytes is one
    // kernel, the 4-byte tail of an odd size was a second one, ~5 us per sort)
    if (zero_joint && hipMemsetAsync(joint, 0, (size_t)kJointBins * kJointBins * 4 + 16, s) != hipSuccess)
        return RSORT_ERR_HIP;
    return hip_status(launch_histogram_joint(a, s));
}

// The next pass's chunks from the joint counts (rs_joint_bounds), after this pass's table is scanned
// (ctab: a cut plan's pieces become row tasks where every chunk wrote its rows).
int do_joint_bounds(const rsort_plan &p, const uint32_t *joint, const uint32_t *enable, uint32_t *bounds,
                    uint32_t *plan, uint32_t *pcounts, const uint32_t *ctab, uint32_t *rows_cnt,
                    const uint32_t *rowone, hipStream_t s) {
    PhaseScope ps(RSORT_PHASE_HISTOGRAM, p.n, s);
    // a group may take one tile more than a fixed chunk; a cut-plan chunk boundary moves to a
    // group boundary up to half a tile (and a quarter chunk) away
    const uint32_t snap = (uint32_t)std::min<int64_t>(p.tile_keys / 2, p.n / (4 * (int64_t)kJointBins));
    // the first cut plan of a sort (pass 1's, from pass 0's joint counts) balances estimated cost
    // (rs_joint_bounds; RSORT_CUT_WEIGHTS=0 turns it off for A/B runs)
    const uint32_t weighted = (enable == nullptr && cut_weights()) ? 1u : 0u;
    return hip_status(launch_joint_bounds(joint, enable, bounds, plan, pcounts, (uint64_t)p.n,
                                          (uint64_t)p.chunk_keys + (uint64_t)p.tile_keys, snap, weighted, s,
                                          ctab, rows_cnt, rowone));
}

int do_histogram(const rsort_plan &p, const uint32_t *keys, int shift, uint32_t *table,
                 int dmode, const uint32_t *split, int nsplit, hipStream_t s,
                 const uint32_t *bounds = nullptr, uint32_t *copy_src = nullptr,
                 const uint32_t *plan = nullptr, uint32_t *pcounts = nullptr, uint32_t *zero = nullptr,
                 uint32_t *done = nullptr, uint32_t *rows = nullptr) {
    HistArgs a{};
    a.rows = rows;
    a.zero = zero;
    a.zero_n = zero ? (uint64_t)p.table_entries : 0u;
    a.done = done;
    a.bounds = bounds;
    a.copy_src = copy_src;
    a.plan = plan;
    a.pcounts = pcounts;
    a.keys = keys;
    a.table = table;
    a.n = (uint64_t)p.n;
    a.chunk_keys = (uint64_t)p.chunk_keys;
    a.num_chunks = (uint32_t)p.num_chunks;
    a.shift = (uint32_t)shift;
    a.vec = (((uintptr_t)keys & 15u) == 0) ? 1u : 0u;
    a.nsplit = (uint32_t)nsplit;
    for (int i = 0; i < nsplit; ++i) a.splitters[i] = split[i];
    // few, long chunks (one scatter workgroup per CU): several histogram workgroups per chunk,
    // their counts added into a zeroed table
    const int cus = device_cus();
    const int64_t want = 4 * (int64_t)(cus > 0 ? cus : 256);  // 1024-thread workgroups (hist_bits)
    a.split = 1;
    if (bounds != nullptr) {
        // a digit-group pass (256 chunks of one workgroup each): copies the joint counts, counts the
        // cut plan's pieces, or counts one chunk per 1024-thread workgroup (as fast as split
        // workgroups, 0.62 ms per 2^30 keys, and no table memset launch)
        a.wide = 1;
    } else if (p.num_chunks < want && p.chunk_keys >= 8 * 4096) {
        a.split = (uint32_t)std::min<int64_t>({(want + p.num_chunks - 1) / p.num_chunks, p.chunk_keys / 4096, 64});
    }
    PhaseScope ps(RSORT_PHASE_HISTOGRAM, p.n, s);
    if (a.split > 1 && hipMemsetAsync(table, 0, (size_t)p.table_entries * 4, s) != hipSuccess) return RSORT_ERR_HIP;
    return hip_status(launch_histogram(p.k_bits, dmode, a, s));
}

int do_scan(const rsort_plan &p, uint32_t *table, uint32_t *bsums, hipStream_t s, uint32_t *zero = nullptr,
            uint32_t *done = nullptr, const Carve *cut = nullptr, const uint32_t *group_flag = nullptr) {
    ScanArgs a{};
    a.done = done;
    if (cut != nullptr) {
        // a digit-group pass: under a cut plan the scan assembles the table first
        a.group_flag = group_flag;
        a.joint = cut->joint;
        a.plan = cut->plan;
        a.pcounts = cut->pcounts;
    }
    a.table = table;
    a.block_sums = bsums;
    a.zero = zero;
    a.zero_n = zero ? (uint64_t)p.table_entries : 0u;
    a.m = (uint64_t)p.table_entries;
    a.nblocks = (uint32_t)p.scan_blocks;
    PhaseScope ps(RSORT_PHASE_SCAN, p.table_entries, s);
    return hip_status(launch_scan(a, s));
}

int do_scatter(const rsort_plan &p, const uint32_t *kin, const uint32_t *vin, uint32_t *kout,
               uint32_t *vout, int shift, const uint32_t *table, int local_only, int dmode,
               const uint32_t *split, int nsplit, hipStream_t s, const uint32_t *bounds = nullptr,
               uint32_t *next_table = nullptr, uint32_t *tail_zero = nullptr, uint32_t *done = nullptr,
               const uint32_t *cl_select = nullptr, int raw_table = 0, uint32_t *zero_table = nullptr,
               uint32_t *check = nullptr) {
    ScatterArgs a{};
    a.check = check;
    a.rank_fault = g_rank_fault.load() ? 1u : 0u;
    a.raw_table = raw_table ? 1u : 0u;
    a.zero_table = zero_table;
    a.cl_select = cl_select;
    a.bounds = bounds;
    a.next_table = next_table;
    a.tail_zero = tail_zero;
    a.done = done;
    a.kin = kin;
    a.vin = vin;
    a.kout = kout;
    a.vout = vout;
    a.table = table;
    a.n = (uint64_t)p.n;
    a.chunk_keys = (uint64_t)p.chunk_keys;
    a.num_chunks = (uint32_t)p.num_chunks;
    a.shift = (uint32_t)shift;
    a.local_only = local_only ? 1u : 0u;
    a.nsplit = (uint32_t)nsplit;
    for (int i = 0; i < nsplit; ++i) a.splitters[i] = split[i];
    const int rank = internal_rank((dmode == kDigitShift) ? g_rank_algo.load() : RSORT_RANK_MATCH);
    const int geom = geom_from_shape(p.threads, p.tile_keys, p.pairs);
    if (!scatter_available(p.k_bits, p.pairs, rank, dmode, geom)) return RSORT_ERR_ARG;
    const int aligned16 = line_capable(kout, vout, p.pairs, p.n);
    if ((bounds || next_table || raw_table) && !(rank == kRankAtomic && aligned16 && !local_only && dmode == kDigitShift))
        return RSORT_ERR_ARG;  // group chunks, next-digit counts, raw tables: rs_scatter_lines only
    // a multi-GPU partition's scatter (splitter digits) is recorded apart from the sort's passes
    PhaseScope ps(dmode == kDigitSplit ? RSORT_PHASE_PARTITION : RSORT_PHASE_SCATTER, p.n, s);
    return hip_status(launch_scatter(p.k_bits, p.pairs, rank, dmode, geom, local_only ? 0 : aligned16, a, s));
}

int check_plan(const rsort_plan *p) {
    if (!p) return RSORT_ERR_ARG;
    if (p->k_bits < kMinBits || p->k_bits > kMaxBits) return RSORT_ERR_BITS;
    if (p->n < 0 || p->n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (geom_from_shape(p->threads, p->tile_keys, p->pairs) < 0) return RSORT_ERR_ARG;
    if (p->tiles_per_chunk <= 0 || p->num_chunks <= 0 ||
        p->num_chunks * p->tiles_per_chunk * p->tile_keys < p->n ||
        p->chunk_keys != p->tiles_per_chunk * p->tile_keys || p->bins != (1 << p->k_bits) ||
        p->table_entries != (int64_t)p->bins * p->num_chunks)
        return RSORT_ERR_ARG;
    return RSORT_OK;
}

int sort_planned(const rsort_plan &p, const uint32_t *kin, const uint32_t *vin, uint32_t *kout,
                 uint32_t *vout, void *ws, size_t wsb, hipStream_t s) {
    int st = check_plan(&p);
    if (st) return st;
    if (p.n == 0) return RSORT_OK;
    if (!kin || !kout || !ws || (p.pairs && (!vin || !vout))) return RSORT_ERR_ARG;
    if (!aligned4(kin) || !aligned4(kout) || (p.pairs && (!aligned4(vin) || !aligned4(vout))))
        return RSORT_ERR_ALIGN;
    if (wsb < p.workspace_bytes) return RSORT_ERR_WORKSPACE;
    const Carve c = carve(p, ws);
    const int P = p.passes;
    const uint32_t *sk = kin, *sv = vin;
    const bool inplace = (kin == kout) || (p.pairs && vin == vout);
    if (inplace && (P % 2 == 1)) {
        // pass 0 must not read the buffer it writes: stage the input in the ping-pong buffer
        PhaseScope ps(RSORT_PHASE_COPY, p.n, s);
        if (hipMemcpyAsync(c.tmp_k, kin, (size_t)p.n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return RSORT_ERR_HIP;
        if (p.pairs &&
            hipMemcpyAsync(c.tmp_v, vin, (size_t)p.n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return RSORT_ERR_HIP;
        sk = c.tmp_k;
        sv = c.tmp_v;
    }
    // digit-group chunks on every second pass (joint_plan): needs rs_scatter_lines for both
    // outputs (lane-ordered ranks, 16-B aligned ping-pong buffers)
    const bool joint = joint_plan(p) && g_group_chunks.load() != 0 &&
                       internal_rank(g_rank_algo.load()) == kRankAtomic && line_capable(kout, vout, p.pairs, p.n) &&
                       line_capable(c.tmp_k, c.tmp_v, p.pairs, p.n);
    if (joint_plan(p) && !joint &&
        hipMemsetAsync(c.bounds, 0, (size_t)2 * kBoundsWords * 4, s) != hipSuccess)  // rsort_group_flags: none
        return RSORT_ERR_HIP;
    // next-digit counts (k = 3, 4): the same kernel conditions as digit groups
    const bool nextc = next_plan(p) && g_group_chunks.load() != 0 && internal_rank(g_rank_algo.load()) == kRankAtomic &&
                       line_capable(kout, nullptr, 0, p.n) && line_capable(c.tmp_k, nullptr, 0, p.n);
    // next-digit plans: every pass after the first derives its offsets from the raw counts the pass
    // before added (three tables in rotation: read / added into / cleared for the pass after next),
    // instead of the last workgroup of each pass scanning them (RSORT_NX_TAIL=1: that older way)
    // (raw tables only up to kRawTableMaxChunks chunks: each workgroup reads the whole table)
    const bool rawt = nextc && !nx_tail() && p.num_chunks <= kRawTableMaxChunks;
    uint32_t *const rot[3] = {c.table, c.table2, c.table3};
    uint32_t *const rows = piece_rows() ? c.rows : nullptr, *const rows_cnt = rows ? c.rows_cnt : nullptr;
    for (int i = 0; i < P; ++i) {
        const int shift = i * p.k_bits;
        const bool to_out = ((P - 1 - i) % 2) == 0;  // the last pass always lands in `out`
        uint32_t *dk = to_out ? kout : c.tmp_k;
        uint32_t *dv = to_out ? vout : c.tmp_v;
        // even pass i counts the joint counts for pass i + 1; odd pass i may use them
        const bool count_joint = joint && (i % 2 == 0) && i + 1 < P;
        const uint32_t *bounds = (joint && (i % 2 == 1)) ? c.bounds + (i / 2) * kBoundsWords : nullptr;
        // next-digit plans alternate two tables (tail scans) or rotate three (raw tables): pass i
        // reads tab, adds pass i + 1's into nxt
        uint32_t *tab = rawt ? rot[i % 3] : (nextc && (i % 2 == 1)) ? c.table2 : c.table;
        uint32_t *nxt = (nextc && i + 1 < P) ? (rawt ? rot[(i + 1) % 3] : (i % 2 == 1) ? c.table : c.table2) : nullptr;
        uint32_t *clr = (rawt && i + 2 < P) ? rot[(i + 2) % 3] : nullptr;  // for the pass after next
        const uint32_t *enable = (count_joint && i >= 2) ? c.bounds + (i / 2 - 1) * kBoundsWords : nullptr;
        // pass 0's histogram clears the check words (rsort_plan_check: a clean record for this sort)
        if (count_joint) {
            if ((st = do_histogram_joint(p, sk, shift, c.table, c.joint, enable, s, i == 0, rows, rows_cnt,
                                         i == 0 ? c.done : nullptr)))
                return st;
        } else if (!(nextc && i > 0) &&
                   (st = do_histogram(p, sk, shift, tab, kDigitShift, nullptr, 0, s, bounds, c.joint, c.plan,
                                      c.pcounts, rawt ? nxt : nullptr, i == 0 ? c.done : nullptr,
                                      bounds ? rows : nullptr))) {
            return st;
        }
        // next-digit plans: pass 0's table is scanned by launches (which also arm the tail counter;
        // raw tables: no scan at all, the histogram cleared the next table), every later table by the
        // previous scatter's last workgroup (raw tables: by every workgroup of the pass itself)
        if (!(nextc && i > 0) && !rawt &&
            (st = do_scan(p, tab, c.bsums, s, nxt, nextc ? c.done : nullptr, bounds ? &c : nullptr, bounds)))
            return st;
        // the next pass's chunks (after the scan: a cut plan finds the previous chunks' positions in it)
        if (count_joint && (st = do_joint_bounds(p, c.joint, enable, c.bounds + (i / 2) * kBoundsWords, c.plan,
                                                 c.pcounts, tab, rows_cnt, rows ? rows + kRowsWords : nullptr, s)))
            return st;
        // passes after the first of a digit-group sort: where the previous odd pass's groups were
        // unbalanced (skewed, duplicate-heavy keys: runs of equal keys in this pass's input), the
        // clustered-input kernel runs (rank_add_hot), else the plain one -- chosen on the device
        const uint32_t *cl = (joint && i >= 1) ? c.bounds + ((i - 1) / 2) * kBoundsWords : nullptr;
        if ((st = do_scatter(p, sk, sv, dk, dv, shift, tab, 0, kDigitShift, nullptr, 0, s, bounds, nxt,
                             (nxt && !rawt) ? tab : nullptr, (nextc && (nxt || rawt)) ? c.done : nullptr, cl,
                             rawt, clr, c.done + kDoneErr)))
            return st;
        // test hook: corrupt the raw table pass 1 reads (its total is then not n: every pass-1 workgroup
        // writes nothing and records the failure for rsort_plan_check / RSORT_ERR_CHECK)
        if (i == 0 && rawt && nxt && g_table_fault.load() &&
            hipMemsetD32Async((hipDeviceptr_t)nxt, 0xFFFFFFFFu, 1, s) != hipSuccess)
            return RSORT_ERR_HIP;
        sk = dk;
        sv = dv;
    }
    return RSORT_OK;
}

// ------------------------------------------------------------------------------ host entry cache
struct DevCache {
    std::mutex mu;
    int device = -1;
    void *buf = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
};
std::mutex g_cache_mu;
std::vector<DevCache *> g_caches;

DevCache *cache_for(int dev) {
    std::lock_guard<std::mutex> g(g_cache_mu);
    for (DevCache *c : g_caches)
        if (c->device == dev) return c;
    DevCache *c = new DevCache();
    c->device = dev;
    g_caches.push_back(c);
    return c;
}

int host_sort(const uint32_t *kin, const uint32_t *vin, uint32_t *kout, uint32_t *vout,
              int64_t n, int k, rsort_phase_times *times) {
    const int pairs = vin != nullptr;
    rsort_plan p;
    int st = plan_fill(n, k, pairs, 0, &p);
    if (st) return st;
    if (n == 0) {
        if (times) memset(times, 0, sizeof(*times));
        return RSORT_OK;
    }
    if (!kin || !kout || (pairs && !vout)) return RSORT_ERR_ARG;
    int count = 0, dev = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return RSORT_ERR_NODEV;
    if (hipGetDevice(&dev) != hipSuccess) return RSORT_ERR_HIP;
    DevCache *dc = cache_for(dev);
    std::lock_guard<std::mutex> g(dc->mu);
    const size_t nb = align256((size_t)n * 4);
    const size_t need = nb * (pairs ? 4 : 2) + p.workspace_bytes;
    if (!dc->stream && hipStreamCreateWithFlags(&dc->stream, hipStreamNonBlocking) != hipSuccess)
        return RSORT_ERR_HIP;
    if (dc->cap < need) {
        if (dc->buf) (void)hipFree(dc->buf);
        dc->buf = nullptr;
        dc->cap = 0;
        if (hipMalloc(&dc->buf, need) != hipSuccess) return RSORT_ERR_ALLOC;
        dc->cap = need;
    }
    char *q = (char *)dc->buf;
    uint32_t *d_kin = (uint32_t *)q;
    uint32_t *d_kout = (uint32_t *)(q + nb);
    uint32_t *d_vin = pairs ? (uint32_t *)(q + 2 * nb) : nullptr;
    uint32_t *d_vout = pairs ? (uint32_t *)(q + 3 * nb) : nullptr;
    void *ws = q + nb * (pairs ? 4 : 2);
    hipStream_t s = dc->stream;
    if (hipMemcpyAsync(d_kin, kin, (size_t)n * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return RSORT_ERR_HIP;
    if (pairs && hipMemcpyAsync(d_vin, vin, (size_t)n * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return RSORT_ERR_HIP;
    if (times) rsort_profile_begin();
    st = sort_planned(p, d_kin, d_vin, d_kout, d_vout, ws, p.workspace_bytes, s);
    if (times) {
        const int st2 = rsort_profile_end(times);
        if (!st) st = st2;
    }
    if (st) {
        (void)hipStreamSynchronize(s);
        return st;
    }
    if (hipMemcpyAsync(kout, d_kout, (size_t)n * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return RSORT_ERR_HIP;
    if (pairs && hipMemcpyAsync(vout, d_vout, (size_t)n * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return RSORT_ERR_HIP;
    // this entry waits for the device anyway: the sort's self-checks (rsort_plan_check) are read here
    uint32_t check = 0;
    if (hipMemcpyAsync(&check, carve(p, ws).done + kDoneErr, 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    return check ? RSORT_ERR_CHECK : RSORT_OK;
}

}  // namespace

void rsort::profile_pause(int delta) { t_prof_paused += delta; }

// ================================================================================ C ABI
extern "C" {

const char *rsort_status_string(int status) {
    switch (status) {
        case RSORT_OK: return "ok";
        case RSORT_ERR_ARG: return "invalid argument";
        case RSORT_ERR_BITS: return "k_bits outside [1, 13]";
        case RSORT_ERR_SIZE: return "n outside [0, 2^32)";
        case RSORT_ERR_ALIGN: return "device buffer not 4-byte aligned";
        case RSORT_ERR_ALLOC: return "allocation failed";
        case RSORT_ERR_HIP: return "HIP runtime error";
        case RSORT_ERR_WORKSPACE: return "workspace too small";
        case RSORT_ERR_NODEV: return "no HIP device";
        case RSORT_ERR_CAPACITY: return "output capacity too small for the received keys";
        case RSORT_ERR_COMM: return "RCCL communication error";
        case RSORT_ERR_CHECK: return "an on-device self-check of the sort failed";
        default: return "unknown status";
    }
}

int rsort_version(void) { return kVersion; }

int rsort_plan_make(int64_t n, int k_bits, int pairs, int64_t tiles_per_chunk, rsort_plan *plan) {
    return plan_fill(n, k_bits, pairs, tiles_per_chunk, plan);
}

size_t rsort_workspace_size(int64_t n, int k_bits, int pairs) {
    rsort_plan p;
    if (plan_fill(n, k_bits, pairs, 0, &p) != RSORT_OK) return 0;
    return p.workspace_bytes;
}

int rsort_sort_planned(const rsort_plan *plan, const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                       uint32_t *d_keys_out, uint32_t *d_vals_out, void *d_workspace,
                       size_t workspace_bytes, void *stream) {
    if (!plan) return RSORT_ERR_ARG;
    return sort_planned(*plan, d_keys_in, d_vals_in, d_keys_out, d_vals_out, d_workspace,
                        workspace_bytes, (hipStream_t)stream);
}

int rsort_u32_device(const uint32_t *d_in, uint32_t *d_out, int64_t n, int k_bits,
                     void *d_workspace, size_t workspace_bytes, void *stream) {
    rsort_plan p;
    const int st = plan_fill(n, k_bits, 0, 0, &p);
    if (st) return st;
    return sort_planned(p, d_in, nullptr, d_out, nullptr, d_workspace, workspace_bytes,
                        (hipStream_t)stream);
}

int rsort_u32_pairs_device(const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                           uint32_t *d_keys_out, uint32_t *d_vals_out, int64_t n, int k_bits,
                           void *d_workspace, size_t workspace_bytes, void *stream) {
    rsort_plan p;
    const int st = plan_fill(n, k_bits, 1, 0, &p);
    if (st) return st;
    return sort_planned(p, d_keys_in, d_vals_in, d_keys_out, d_vals_out, d_workspace,
                        workspace_bytes, (hipStream_t)stream);
}

int rsort_u32(const uint32_t *in, uint32_t *out, int64_t n, int k_bits) {
    return host_sort(in, nullptr, out, nullptr, n, k_bits, nullptr);
}

int rsort_u32_ex(const uint32_t *in, uint32_t *out, int64_t n, int k_bits, int block_size,
                 rsort_phase_times *times) {
    (void)block_size;
    return host_sort(in, nullptr, out, nullptr, n, k_bits, times);
}

int rsort_u32_pairs(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *keys_out,
                    uint32_t *vals_out, int64_t n, int k_bits) {
    if (n > 0 && (!vals_in || !vals_out)) return RSORT_ERR_ARG;
    return host_sort(keys_in, vals_in, keys_out, vals_out, n, k_bits, nullptr);
}

int rsort_pass_histogram(const rsort_plan *plan, const uint32_t *d_keys, int shift,
                         uint32_t *d_table, void *stream) {
    int st = check_plan(plan);
    if (st) return st;
    if (shift < 0 || shift > 31) return RSORT_ERR_ARG;
    if (plan->n == 0) return RSORT_OK;
    if (!d_keys || !d_table) return RSORT_ERR_ARG;
    return do_histogram(*plan, d_keys, shift, d_table, kDigitShift, nullptr, 0, (hipStream_t)stream);
}

int rsort_pass_scan(const rsort_plan *plan, uint32_t *d_table, uint32_t *d_block_sums, void *stream) {
    int st = check_plan(plan);
    if (st) return st;
    if (plan->n == 0) return RSORT_OK;
    if (!d_table || !d_block_sums) return RSORT_ERR_ARG;
    return do_scan(*plan, d_table, d_block_sums, (hipStream_t)stream);
}

int rsort_pass_scatter(const rsort_plan *plan, const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                       uint32_t *d_keys_out, uint32_t *d_vals_out, int shift, const uint32_t *d_table,
                       void *stream) {
    int st = check_plan(plan);
    if (st) return st;
    if (shift < 0 || shift > 31) return RSORT_ERR_ARG;
    if (plan->n == 0) return RSORT_OK;
    if (!d_keys_in || !d_keys_out || !d_table || (plan->pairs && (!d_vals_in || !d_vals_out)))
        return RSORT_ERR_ARG;
    return do_scatter(*plan, d_keys_in, d_vals_in, d_keys_out, d_vals_out, shift, d_table, 0,
                      kDigitShift, nullptr, 0, (hipStream_t)stream);
}

int rsort_pass_local_sort(const rsort_plan *plan, const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                          uint32_t *d_keys_out, uint32_t *d_vals_out, int shift, void *stream) {
    int st = check_plan(plan);
    if (st) return st;
    if (shift < 0 || shift > 31) return RSORT_ERR_ARG;
    if (plan->n == 0) return RSORT_OK;
    if (!d_keys_in || !d_keys_out || (plan->pairs && (!d_vals_in || !d_vals_out)))
        return RSORT_ERR_ARG;
    if (d_keys_in == d_keys_out) return RSORT_ERR_ARG;
    // local-only mode never reads the offset table
    const uint32_t *table = nullptr;
    return do_scatter(*plan, d_keys_in, d_vals_in, d_keys_out, d_vals_out, shift, table, 1,
                      kDigitShift, nullptr, 0, (hipStream_t)stream);
}

int rsort_set_rank_algo(int algo) {
    if (algo != RSORT_RANK_MATCH && algo != RSORT_RANK_SPLIT && algo != RSORT_RANK_BALLOT) return RSORT_ERR_ARG;
    g_rank_algo.store(algo);
    return RSORT_OK;
}

int rsort_get_rank_algo(void) { return g_rank_algo.load(); }

int rsort_set_group_chunks(int enable) {
    g_group_chunks.store(enable ? 1 : 0);
    return RSORT_OK;
}

int rsort_get_group_chunks(void) { return g_group_chunks.load(); }

int rsort_group_flags(const rsort_plan *plan, const void *d_workspace, int *flags, void *stream) {
    if (!plan || !flags || !d_workspace) return RSORT_ERR_ARG;
    int st = check_plan(plan);
    if (st) return st;
    flags[0] = flags[1] = 0;
    if (!joint_plan(*plan) || plan->n == 0) return RSORT_OK;
    const Carve c = carve(*plan, const_cast<void *>(d_workspace));
    hipStream_t s = (hipStream_t)stream;
    uint32_t h[2] = {0, 0};
    for (int i = 0; i < 2; ++i)
        if (2 * i + 1 < plan->passes &&
            hipMemcpyAsync(&h[i], c.bounds + i * kBoundsWords, 4, hipMemcpyDeviceToHost, s) != hipSuccess)
            return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    flags[0] = (int)h[0];  // kGroupsFixed / kGroupsWhole / kGroupsCut
    flags[1] = (int)h[1];
    return RSORT_OK;
}

int rsort_cut_plan_stats(const rsort_plan *plan, const void *d_workspace, int *stats, void *stream) {
    if (!plan || !stats || !d_workspace) return RSORT_ERR_ARG;
    int st = check_plan(plan);
    if (st) return st;
    for (int i = 0; i < 8; ++i) stats[i] = 0;
    if (!joint_plan(*plan) || plan->n == 0) return RSORT_OK;
    const Carve c = carve(*plan, const_cast<void *>(d_workspace));
    hipStream_t s = (hipStream_t)stream;
    uint32_t h[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int i = 0; i < 2; ++i)
        if (2 * i + 1 < plan->passes &&
            hipMemcpyAsync(h[i], c.bounds + i * kBoundsWords + kBoundsStat, 16, hipMemcpyDeviceToHost, s) != hipSuccess)
            return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 4; ++j) stats[4 * i + j] = (int)h[i][j];
    return RSORT_OK;
}

int rsort_plan_features(const rsort_plan *plan) {
    if (check_plan(plan) != RSORT_OK) return -RSORT_ERR_ARG;
    const rsort_plan &p = *plan;
    const bool atomic = internal_rank(g_rank_algo.load()) == kRankAtomic;
    const bool on = g_group_chunks.load() != 0 && atomic;
    int f = 0;
    if (joint_plan(p) && on) f |= RSORT_FEAT_GROUPS;
    if (next_plan(p) && on) {
        f |= RSORT_FEAT_NEXT_DIGIT;
        f |= (!nx_tail() && p.num_chunks <= kRawTableMaxChunks) ? RSORT_FEAT_RAW_TABLES : RSORT_FEAT_TAIL_SCAN;
    }
    return f;
}

int rsort_inject_table_fault(int enable) { return g_table_fault.exchange(enable ? 1 : 0); }

int rsort_inject_rank_fault(int enable) { return g_rank_fault.exchange(enable ? 1 : 0); }

int rsort_plan_check(const rsort_plan *plan, const void *d_workspace, int *flags, void *stream) {
    if (!plan || !flags || !d_workspace) return RSORT_ERR_ARG;
    int st = check_plan(plan);
    if (st) return st;
    *flags = 0;
    if (plan->n == 0) return RSORT_OK;
    const Carve c = carve(*plan, const_cast<void *>(d_workspace));
    hipStream_t s = (hipStream_t)stream;
    uint32_t h = 0;
    if (hipMemcpyAsync(&h, c.done + kDoneErr, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    *flags = (int)(h & (kCheckTable | kCheckRankOrder));
    return RSORT_OK;
}

size_t rsort_scatter_kernels_used(char *buf, size_t len, int reset) {
    return scatter_kernels_used(buf, len, reset);
}

int rsort_lane_order_probe(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return -RSORT_ERR_NODEV;
    return lane_order_probe();
}

int rsort_profile_begin(void) {
    std::lock_guard<std::mutex> g(g_prof.mu);
    for (auto &r : g_prof.recs) {
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.recs.clear();
    g_prof.on = true;
    return RSORT_OK;
}

int rsort_profile_end(rsort_phase_times *out) {
    std::vector<ProfRec> recs;
    {
        std::lock_guard<std::mutex> g(g_prof.mu);
        g_prof.on = false;
        recs.swap(g_prof.recs);
    }
    rsort_phase_times t;
    memset(&t, 0, sizeof(t));
    int st = RSORT_OK;
    for (auto &r : recs) {
        if (hipEventSynchronize(r.b) != hipSuccess) {
            st = RSORT_ERR_HIP;
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
            st = RSORT_ERR_HIP;
            continue;
        }
        t.ms[r.phase] += ms;
        t.launches[r.phase] += 1;
        t.keys[r.phase] += r.keys;
    }
    {
        std::lock_guard<std::mutex> g(g_prof.mu);
        for (auto &r : recs) {
            g_prof.pool.push_back(r.a);
            g_prof.pool.push_back(r.b);
        }
    }
    if (out) *out = t;
    return st;
}

size_t rsort_partition_workspace_size(int64_t n, int num_buckets, int pairs) {
    if (num_buckets < 1 || num_buckets > kMaxSplitters + 1) return 0;
    const int bits = partition_bits(n, num_buckets, pairs);
    rsort_plan p;
    if (plan_fill(n, bits, pairs, 0, &p, /*partition=*/1) != RSORT_OK) return 0;
    return p.workspace_bytes;
}

int rsort_partition_device(const uint32_t *d_keys_in, const uint32_t *d_vals_in, uint32_t *d_keys_out,
                           uint32_t *d_vals_out, int64_t n, const uint32_t *splitters, int num_buckets,
                           uint32_t *d_bucket_starts, void *d_workspace, size_t workspace_bytes,
                           void *stream) {
    if (num_buckets < 1 || num_buckets > kMaxSplitters + 1) return RSORT_ERR_ARG;
    if (num_buckets > 1 && !splitters) return RSORT_ERR_ARG;
    for (int i = 1; i + 1 < num_buckets; ++i)
        if (splitters[i] < splitters[i - 1]) return RSORT_ERR_ARG;
    const int pairs = d_vals_in != nullptr;
    const int bits = partition_bits(n < 0 ? 0 : n, num_buckets, pairs);
    rsort_plan p;
    int st = plan_fill(n, bits, pairs, 0, &p, /*partition=*/1);
    if (st) return st;
    if (!d_bucket_starts) return RSORT_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        return hip_status(hipMemsetAsync(d_bucket_starts, 0, (size_t)(num_buckets + 1) * 4, s));
    }
    if (!d_keys_in || !d_keys_out || !d_workspace || (pairs && !d_vals_out)) return RSORT_ERR_ARG;
    if (d_keys_in == d_keys_out) return RSORT_ERR_ARG;
    if (workspace_bytes < p.workspace_bytes) return RSORT_ERR_WORKSPACE;
    const Carve c = carve(p, d_workspace);
    const int ns = num_buckets - 1;
    // (the check words as a sort's: cleared by the histogram, the scatter's rank check recorded there)
    if ((st = do_histogram(p, d_keys_in, 0, c.table, kDigitSplit, splitters, ns, s, nullptr, nullptr, nullptr,
                           nullptr, nullptr, c.done)))
        return st;
    if ((st = do_scan(p, c.table, c.bsums, s))) return st;
    if ((st = do_scatter(p, d_keys_in, d_vals_in, d_keys_out, d_vals_out, 0, c.table, 0, kDigitSplit,
                         splitters, ns, s, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr,
                         c.done + kDoneErr)))
        return st;
    return hip_status(launch_gather_starts(c.table, (uint32_t)p.num_chunks, (uint32_t)num_buckets,
                                           (uint64_t)n, d_bucket_starts, s));
}

int rsort_partition_check(int64_t n, int num_buckets, int pairs, const void *d_workspace, int *flags, void *stream) {
    if (!flags || !d_workspace || num_buckets < 1 || num_buckets > kMaxSplitters + 1) return RSORT_ERR_ARG;
    *flags = 0;
    rsort_plan p;
    int st = plan_fill(n < 0 ? 0 : n, partition_bits(n < 0 ? 0 : n, num_buckets, pairs ? 1 : 0), pairs ? 1 : 0, 0, &p,
                       /*partition=*/1);
    if (st) return st;
    if (n <= 0) return RSORT_OK;
    const Carve c = carve(p, const_cast<void *>(d_workspace));
    hipStream_t s = (hipStream_t)stream;
    uint32_t h = 0;
    if (hipMemcpyAsync(&h, c.done + kDoneErr, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    *flags = (int)(h & (kCheckTable | kCheckRankOrder));
    return RSORT_OK;
}

int rsort_top_histogram(const uint32_t *d_keys, int64_t n, int top_bits, uint32_t *d_hist,
                        void *d_workspace, size_t workspace_bytes, void *stream) {
    rsort_plan p;
    int st = plan_fill(n, top_bits, 0, 0, &p);
    if (st) return st;
    if (!d_hist) return RSORT_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return hip_status(hipMemsetAsync(d_hist, 0, (size_t)p.bins * 4, s));
    if (!d_keys || !d_workspace) return RSORT_ERR_ARG;
    if (workspace_bytes < p.workspace_bytes) return RSORT_ERR_WORKSPACE;
    const Carve c = carve(p, d_workspace);
    if ((st = do_histogram(p, d_keys, 32 - top_bits, c.table, kDigitShift, nullptr, 0, s))) return st;
    if ((st = do_scan(p, c.table, c.bsums, s))) return st;
    hipError_t e = launch_gather_starts(c.table, (uint32_t)p.num_chunks, (uint32_t)p.bins,
                                        (uint64_t)n, c.starts, s);
    if (e != hipSuccess) return RSORT_ERR_HIP;
    return hip_status(launch_diff_starts(c.starts, (uint32_t)p.bins, d_hist, s));
}

int rsort_top_histogram_sampled(const uint32_t *d_keys, int64_t n, int top_bits, int stride, uint32_t *d_hist,
                                void *stream) {
    if (top_bits < 1 || top_bits > kMaxBits) return RSORT_ERR_BITS;
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (stride < 1 || !d_hist || (n > 0 && !d_keys)) return RSORT_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_hist, 0, ((size_t)1 << top_bits) * 4, s) != hipSuccess) return RSORT_ERR_HIP;
    if (n == 0) return RSORT_OK;
    PhaseScope ps(RSORT_PHASE_HISTOGRAM, (n + stride - 1) / stride, s);
    return hip_status(launch_top_hist_sampled(d_keys, (uint64_t)n, (uint32_t)top_bits, (uint32_t)stride, d_hist, s));
}

int rsort_sample_device(const uint32_t *d_keys, int64_t n, int64_t stride, int64_t count, int64_t row_len,
                        uint32_t *d_out, void *stream) {
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (stride < 1 || count < 0 || row_len < count || (row_len > 0 && !d_out) || (count > 0 && n > 0 && !d_keys))
        return RSORT_ERR_ARG;
    return hip_status(launch_sample(d_keys, (uint64_t)n, (uint64_t)stride, (uint64_t)count, (uint64_t)row_len, d_out,
                                    (hipStream_t)stream));
}

int rsort_fingerprint_device(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n, uint64_t *d_out,
                             void *stream) {
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (!d_out || (n > 0 && !d_keys)) return RSORT_ERR_ARG;
    return hip_status(launch_fingerprint(d_keys, d_vals, (uint64_t)n, (unsigned long long *)d_out, (hipStream_t)stream));
}

int rsort_gen_uniform(uint32_t *d_out, int64_t n, uint64_t seed, void *stream) {
    if (n < 0) return RSORT_ERR_SIZE;
    if (n == 0) return RSORT_OK;
    if (!d_out) return RSORT_ERR_ARG;
    return hip_status(launch_gen_uniform(d_out, (uint64_t)n, seed, (hipStream_t)stream));
}

int rsort_gen_zipf(uint32_t *d_out, int64_t n, uint64_t seed, const uint32_t *d_cdf, int64_t ranks,
                   void *stream) {
    if (n < 0) return RSORT_ERR_SIZE;
    if (n == 0) return RSORT_OK;
    if (!d_out || !d_cdf || ranks <= 0) return RSORT_ERR_ARG;
    return hip_status(launch_gen_zipf(d_out, (uint64_t)n, seed, d_cdf, (uint64_t)ranks, (hipStream_t)stream));
}

int rsort_gen_iota(uint32_t *d_out, int64_t n, uint32_t base, void *stream) {
    if (n < 0) return RSORT_ERR_SIZE;
    if (n == 0) return RSORT_OK;
    if (!d_out) return RSORT_ERR_ARG;
    return hip_status(launch_gen_iota(d_out, (uint64_t)n, base, (hipStream_t)stream));
}

}  // extern "C"
