// rsort_internal.hpp -- shared between the HIP kernels (rsort_kernels.hip) and the host
// driver (rsort_capi.cpp). Not part of the public ABI (include/rsort.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace rsort {

constexpr int kWave = 64;
constexpr int kHistThreads = 256;          // workgroup size of the histogram kernel
constexpr int kMinBits = 1;
constexpr int kMaxBits = 13;            // the reference's SMEM limit (Parallel7.cu:740-745)
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 16;
constexpr int kScanSegment = kScanThreads * kScanPerThread;  // table entries per scan block
constexpr int kMaxSplitters = 31;          // partition: <= 32 buckets (2 x 16 ranks' equal-key splitters)

enum DigitMode : int { kDigitShift = 0, kDigitSplit = 1 };

// Scatter-kernel tile geometries (threads x keys per thread). Measured on MI355X at 2^30 keys
// (dev/scatter_lab): the digit runs a tile writes must be long enough to fill 128-B lines, so
// k = 5..8 uses 16384-key tiles; k <= 4 has long runs already; k >= 9 and small inputs use
// 4096-key tiles (LDS for 2^k per-wave counters; enough workgroups to fill 256 CUs).
// kGeomLines (k = 5..8 keys): 16384-key tiles of 1024 threads written as whole 128-B lines
// (rs_scatter_lines; one workgroup per CU, its LDS holds the tile plus every digit's carry).
// kGeomLinesPairs (k = 5..8 pairs): 8192-pair tiles of 1024 threads x 8 (keys + values); k = 7, 8
// through rs_scatter_pairs (128-B lines in both arrays), k = 5, 6 through rs_scatter_lines (64-B lines).
// kGeomXL (k = 13): 4096-key tiles of 128 threads (2 waves), so the 2 x 8192 per-wave counters fit
// in LDS beside the tile (112 KB keys-only).
enum Geom : int { kGeomSmall = 0, kGeomLarge = 1, kGeomK4 = 2, kGeomLines = 3, kGeomLinesPairs = 4, kGeomXL = 5,
                  kGeomCount = 6 };
struct GeomShape {
    int threads;
    int kpt;
};
constexpr GeomShape kGeomShape[kGeomCount] = {{256, 16}, {512, 32}, {512, 16}, {1024, 16}, {1024, 8}, {128, 32}};
// rs_scatter_lines line width. Keys-only stages whole 128-B lines (the L2 line: runs that start or
// end mid-line cost about a third more HBM time, dev/runlen_lab.hip); its pairs instances keep 64-B
// lines (two 128-B carry areas do not fit in LDS beside 8192-key tiles of keys and values) --
// rs_scatter_pairs writes 128-B lines for pairs with its own layout.
constexpr int kLineKeys = 32;
constexpr int kLineKeysPairs = 16;
inline int geom_tile_keys(int g) { return kGeomShape[g].threads * kGeomShape[g].kpt; }
inline int geom_from_shape(int threads, int tile_keys, int pairs) {
    (void)pairs;
    for (int g = 0; g < kGeomCount; ++g)
        if (kGeomShape[g].threads == threads && geom_tile_keys(g) == tile_keys) return g;
    return -1;
}

// Internal ranking variants (rs_scatter's RANK template argument).
// kRankSplit: the reference's 1-bit splits; kRankCount: ballot peer match; kRankAtomic: lane-ordered
// returning LDS adds (the default where rs_lane_order_probe confirms the lane order).
enum RankAlgo : int { kRankSplit = 1, kRankCount = 3, kRankAtomic = 4 };
// Public rsort_rank_algo -> internal variant for the current device (probes lane order once).
int internal_rank(int public_algo);
// 1 / 0: same-address ds_add_rtn lanes are served in lane order on the current device; < 0 error.
int lane_order_probe();

struct HistArgs {
    const uint32_t *keys;
    uint32_t *table;        // [bins][num_chunks]
    uint64_t n;
    uint64_t chunk_keys;
    uint32_t num_chunks;
    uint32_t shift;
    uint32_t vec;           // keys 16-byte aligned: uint4 loads
    uint32_t split;         // workgroups per chunk (> 1: partial counts added into a zeroed table)
    uint32_t nsplit;
    uint32_t splitters[kMaxSplitters];
    // Digit-group chunks (kJointBits plans, see rs_histogram_joint). bounds != nullptr and
    // bounds[0] == kGroupsWhole: this pass's table is copy_src (the previous pass's joint counts),
    // copied instead of counted, and copy_src is cleared as it is read (the next counting pass adds
    // into it). bounds[0] == kGroupsCut: the workgroups count the cut plan's pieces (plan, below)
    // into pcounts; the scan assembles the table.
    const uint32_t *bounds;
    uint32_t *copy_src;
    const uint32_t *plan;
    uint32_t *pcounts;
    uint32_t wide;          // 1: 1024-thread workgroups also with split == 1 (one per chunk, no memset)
    // rs_histogram_joint only: the joint counts [next digit][digit] are added into `joint`
    // (zeroed); joint_enable == nullptr or *joint_enable != kGroupsFixed turns the joint count on.
    uint32_t *joint;
    const uint32_t *joint_enable;
    // raw-table next-digit plans (k = 3, 4), pass 0: the histogram also clears `zero` (zero_n words: the
    // table pass 0's scatter counts into) and the check words done[0], done[kDoneErr]; its table is
    // then read raw by the scatter (ScatterArgs::raw_table), with no scan launches
    uint32_t *zero;
    uint64_t zero_n;
    uint32_t *done;
    // joint-count histograms: != nullptr -> a workgroup whose chunk is skewed (a digit holds more
    // than twice its share) or that follows a cut plan (*joint_enable == kGroupsCut) also writes its
    // joint counts as rows[c][digit][next digit] (R x R words per chunk) and bumps *rows_cnt; a cut
    // plan made when every chunk wrote them takes its pieces' counts from the rows (rs_joint_bounds).
    // Piece-mode launches: the rows the plan's row tasks sum.
    uint32_t *rows;
    uint32_t *rows_cnt;
};

struct ScatterArgs {
    const uint32_t *kin;
    const uint32_t *vin;
    uint32_t *kout;
    uint32_t *vout;
    const uint32_t *table;  // scanned [bins][num_chunks]
    uint64_t n;
    uint64_t chunk_keys;
    uint32_t num_chunks;
    uint32_t shift;
    uint32_t local_only;    // 1: write each tile's local order back in place of the tile
    uint32_t nsplit;
    uint32_t splitters[kMaxSplitters];
    unsigned long long *stamps;  // unused by the library; dev/lines_exp.hip's per-phase cycle stamps
    // rs_scatter_lines only: bounds != nullptr and bounds[0] != 0 -> chunk c is the key range
    // [bounds[1 + c], bounds[2 + c]) (a digit group of the previous pass) instead of
    // [c * chunk_keys, (c + 1) * chunk_keys)
    const uint32_t *bounds;
    // rs_scatter_lines with k <= 4 only: != nullptr -> the next pass's chunk table (zeroed), into
    // which this pass adds every written key's next digit by its destination chunk
    uint32_t *next_table;
    // with next_table: the workgroup that finishes last scans next_table in place (exclusive,
    // the rs_scan_* result), clears tail_zero (the table the next pass counts into; this pass's
    // own, read by every workgroup before it finished) and re-arms *done (zero on entry)
    uint32_t *tail_zero;
    uint32_t *done;
    // k = 8 line kernels: != nullptr -> launch_scatter launches the plain and the clustered-input
    // variant (rank_add_hot); *cl_select == kGroupsWhole runs the plain one, anything else (a pass
    // whose digit groups were unbalanced: skewed, duplicate-heavy keys) the clustered one
    const uint32_t *cl_select;
    // whole-line kernels only (set by launch_scatter): kout / vout are moved down to kout's 128-B-
    // aligned base and every output position up by pos_shift (< 32) keys, so lines are cache lines
    // for any 4-B-aligned output
    uint32_t pos_shift;
    // rs_scatter_lines with k <= 4 (next-digit plans, passes after the first): raw_table = 1 -> `table`
    // holds the previous pass's unscanned counts and every workgroup derives its own offsets from the
    // whole table (no tail scan); done[kDoneErr] is set when the table's total is not n. zero_table:
    // != nullptr -> each workgroup clears its R words of this R x num_chunks table (the one the pass
    // after next counts into)
    uint32_t raw_table;
    uint32_t *zero_table;
    // the lane-ordered kernels (rs_scatter_lines, rs_scatter_pairs, rs_scatter with kRankAtomic): != nullptr ->
    // the sort's check word (done + kDoneErr), where a workgroup whose per-tile rank check failed sets
    // kCheckRankOrder; rank_fault != 0: the test hook that swaps two ranks per digit in every checked slot
    uint32_t *check;
    uint32_t rank_fault;
};

struct ScanArgs {
    uint32_t *table;
    uint32_t *block_sums;
    uint64_t m;             // table entries
    uint32_t nblocks;
    uint32_t *zero;         // optional: zero_n words cleared by the first launch
    uint64_t zero_n;
    uint32_t *done;         // optional: a tail-scan counter (ScatterArgs::done) zeroed by the first launch
    // digit-group plans, odd passes: *group_flag == kGroupsCut -> the first launch assembles the
    // table from the joint counts and the piece counts (cut_entry), the second clears `joint`
    const uint32_t *group_flag;
    uint32_t *joint;
    const uint32_t *plan;
    const uint32_t *pcounts;
};

// Launchers (rsort_kernels.hip). All return hipSuccess or the launch error.
hipError_t launch_histogram(int bits, int dmode, const HistArgs &a, hipStream_t s);
// Digit-group chunks: k = 8 and exactly 2^8 chunks. Pass p counts, besides its own per-chunk
// table, the joint counts of (digit p, digit p + 1) over all keys; pass p + 1's chunks are then
// the digit-p groups of pass p's output, whose per-chunk counts ARE those joint counts, so pass
// p + 1 reads no keys for its histogram.
constexpr int kJointBits = 8;
constexpr uint32_t kJointBins = 1u << kJointBits;
// {flag, chunk starts[0..R], the cut plan's stats}: rs_joint_bounds writes, per odd pass, how its cut plan
// takes its pieces -- key ranges, row tasks (summed joint-count rows), direct adds, negatively counted ranges
// (all 0 for whole groups / fixed chunks); rsort_cut_plan_stats reads them
constexpr uint32_t kBoundsStat = kJointBins + 2;
constexpr uint32_t kBoundsWords = kBoundsStat + 4;
// bounds[0]: how the next pass takes its chunks
//   kGroupsFixed  fixed chunks, histogram counted from the keys (group path off)
//   kGroupsWhole  the digit groups are the chunks (each fits max_keys): table = joint counts
//   kGroupsCut    unbalanced groups (skewed keys): n / R-key chunks, each boundary snapped to a
//                 group boundary within `snap` keys or cutting a group. A cut group's segments
//                 but its largest are counted from the keys ("pieces"), the largest is its
//                 joint column minus the others, every whole group in a chunk is its joint column.
constexpr uint32_t kGroupsFixed = 0, kGroupsWhole = 1, kGroupsCut = 2;
// Cut plan (workspace, rs_joint_bounds): header {key ranges, counted keys, row tasks}, per chunk c a
// descriptor {first group gA | last group gB << 8 | head mode << 16 | tail mode << 18 | empty << 20}
// (head: chunk c's part of gA, slot 2c; tail: its part of gB != gA, slot 2c + 1), per cut group
// {first chunk | last chunk << 8 | derived slot << 16}, the key ranges counted from the keys {start,
// end, slot | kPieceNeg if counted negatively | derived slot << 16, offset among the counted keys}, and
// the row tasks {slot | derived slot << 16, group, first chunk, end chunk} (or direct adds, kRowDirect:
// an end inside a previous chunk whose keys of the group all have one next digit): a counted piece (a cut
// group's part of a chunk, but the group's largest) is the keys of the previous pass's chunks [first,
// end) in that group -- the sum of their joint-count rows (HistArgs::rows) -- plus or minus the keys at
// its two ends (key ranges); without rows the whole piece is one key range. pcounts: kPieceSlots rows
// of R digit counts, one per slot (mod 2^32: a negative range may take a row below zero for a while).
constexpr uint32_t kSegWhole = 0, kSegCounted = 1, kSegDerived = 2;
constexpr uint32_t kPlanDesc = 16;
constexpr uint32_t kPlanGroup = kPlanDesc + kJointBins;
constexpr uint32_t kPlanPieces = kPlanGroup + kJointBins;
constexpr uint32_t kPlanMaxRanges = 4 * kJointBins;  // (<= 255 counted pieces, <= 2 key ranges each)
constexpr uint32_t kPlanRows = kPlanPieces + 4 * kPlanMaxRanges;
constexpr uint32_t kPlanWords = kPlanRows + 4 * 3 * kJointBins;  // (<= 3 tasks per counted piece)
constexpr uint32_t kRowDirect = 0x80000000u;  // row task {slot, kRowDirect | next digit, keys, 0}: a direct add
constexpr uint32_t kPieceSlots = 2 * kJointBins;
constexpr uint32_t kPieceNeg = 0x8000u;  // key range flag (slot word): counted negatively
// joint-count rows: R chunks x R digits x R next digits (64 MiB; then R x R words: each row's one
// next digit, or ~0), and the spills one chunk's rows can hold in LDS (a 16-bit counter spills every
// 2^15 keys: chunk_keys / 2^15 <= 512 at n < 2^32)
constexpr uint64_t kRowsWords = (uint64_t)kJointBins * kJointBins * kJointBins;
constexpr uint32_t kMaxRowSpills = 512;
// Upper bound of what a digit-group plan's workspace holds beyond any other plan's of the same n (the
// joint counts, bounds, cut plan, piece counts and rows, each 256-B aligned): a caller that sizes a
// workspace for one n and sorts a smaller one (the multi-GPU local sort) adds it.
constexpr size_t kJointExtraBytes = ((size_t)kJointBins * kJointBins * 4 + 4 + 255) / 256 * 256 +
                                    ((size_t)2 * kBoundsWords * 4 + 255) / 256 * 256 +
                                    ((size_t)kPlanWords * 4 + 255) / 256 * 256 +
                                    ((size_t)kPieceSlots * kJointBins * 4 + 255) / 256 * 256 +
                                    ((size_t)kRowsWords + kJointBins * kJointBins) * 4;
hipError_t launch_histogram_joint(const HistArgs &a, hipStream_t s);
// From the joint counts [next digit][group]: the next pass's chunks into bounds[1..R+1] and its
// mode into bounds[0] (above): kGroupsWhole when every group fits in max_keys keys, else the cut
// plan (plan, pcounts rows zeroed); kGroupsFixed when the counts do not add up to n or enable
// says the joint count was off (HistArgs::joint_enable). weighted != 0: a cut plan's chunks get
// equal estimated cost instead of equal key counts (rs_joint_bounds).
// ctab: the counting pass's scanned table; rows_cnt: HistArgs::rows_cnt (read and re-armed here);
// rowone: the rows' one-digit words (HistArgs::rows + kRowsWords) -- all given and every chunk's rows
// written: the cut plan's pieces are row tasks + their end keys (or direct adds).
hipError_t launch_joint_bounds(const uint32_t *joint, const uint32_t *enable, uint32_t *bounds,
                               uint32_t *plan, uint32_t *pcounts, uint64_t n, uint64_t max_keys,
                               uint32_t snap, uint32_t weighted, hipStream_t s,
                               const uint32_t *ctab = nullptr, uint32_t *rows_cnt = nullptr,
                               const uint32_t *rowone = nullptr);
// rank_algo: internal RankAlgo. aligned16: the whole-line kernels may run -- keys-only: always
// (any 4-B-aligned kout; launch_scatter shifts positions to kout's 128-B-aligned base); pairs: when
// (vout - kout) % 16 == 0 (otherwise the same plan runs rs_scatter with the same tiles).
hipError_t launch_scatter(int bits, int pairs, int rank_algo, int dmode, int geom, int aligned16,
                          const ScatterArgs &a, hipStream_t s);
// Whether a (bits, pairs, rank_algo, dmode, geom) scatter kernel is compiled in.
bool scatter_available(int bits, int pairs, int rank_algo, int dmode, int geom);
hipError_t launch_scan(const ScanArgs &a, hipStream_t s);
hipError_t launch_gather_starts(const uint32_t *table, uint32_t num_chunks, uint32_t bins,
                                uint64_t n, uint32_t *starts, hipStream_t s);
hipError_t launch_diff_starts(const uint32_t *starts, uint32_t bins, uint32_t *hist,
                              hipStream_t s);
hipError_t launch_top_hist_sampled(const uint32_t *keys, uint64_t n, uint32_t top_bits, uint32_t stride,
                                   uint32_t *hist, hipStream_t s);
hipError_t launch_sample(const uint32_t *keys, uint64_t n, uint64_t stride, uint64_t count, uint64_t row_len,
                         uint32_t *out, hipStream_t s);
hipError_t launch_fingerprint(const uint32_t *keys, const uint32_t *vals, uint64_t n, unsigned long long *out,
                              hipStream_t s);
hipError_t launch_gen_uniform(uint32_t *out, uint64_t n, uint64_t seed, hipStream_t s);
hipError_t launch_gen_zipf(uint32_t *out, uint64_t n, uint64_t seed, const uint32_t *cdf,
                           uint64_t ranks, hipStream_t s);
hipError_t launch_gen_iota(uint32_t *out, uint64_t n, uint32_t base, hipStream_t s);
hipError_t launch_widen(const uint32_t *in, unsigned long long *out, uint32_t n, hipStream_t s);
// Resident scatter workgroups per CU (occupancy query), 0 on error.
int scatter_blocks_per_cu(int bits, int pairs, int rank_algo, int geom, int dmode = kDigitShift);
// Names of the scatter kernel instantiations launched since the last reset, ';'-joined into buf
// (truncated to len - 1 characters); returns the full length. reset != 0 clears the record.
size_t scatter_kernels_used(char *buf, size_t len, int reset);
// rsort_profile_*: while a thread's pause count is > 0 its launches record no phase events (the
// multi-GPU sort's sample sort, which is part of its plan phase, not of the measured passes)
void profile_pause(int delta);
// Workspace check words (every plan: 256 B after the tables): done[0] is the tail-scan counter of next-digit
// plans; done[kDoneErr] is the sort's check word, cleared by pass 0's histogram and read by rsort_plan_check /
// the host entries. Its bits: kCheckTable -- a tail scan or a raw-table pass found a table whose total is not
// n (next-digit plans); kCheckRankOrder -- a lane-ordered scatter kernel's per-tile rank check failed.
constexpr uint32_t kDoneErr = 1;
constexpr uint32_t kCheckTable = 1u, kCheckRankOrder = 2u;
// Raw next-digit tables (every workgroup of a pass sums the whole R x C table for its own starts) cost
// O(R x C) reads per workgroup, O(R x C^2) per pass: only plans of at most this many chunks (about one
// resident wave: C2 has 1024) take them; larger ones keep the tail scan (DESIGN §8 measured
// 2048 chunks 1.155 vs 1.088 ms, 4096 chunks 1.578 vs 1.207 ms per C2 sort against tail scans).
constexpr int64_t kRawTableMaxChunks = 1280;
// Lab switches (A/B runs, dev/lab.sh): the library reads getenv(name) only when RSORT_LAB=1 is set
// too, so a shipped library picks its plans from n, k and the device alone. nullptr otherwise.
inline const char *lab_env(const char *name) {
    const char *lab = getenv("RSORT_LAB");
    if (lab == nullptr || lab[0] != '1') return nullptr;
    return getenv(name);
}

}  // namespace rsort
