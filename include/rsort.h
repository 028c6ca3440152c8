/*
 * rsort.h -- C ABI of the MI355X (gfx950) LSD radix sort (library: cuda.radixsort_amd/librsort.so).
 *
 * Drop-in boundary for the device sort of truongchauhien/CUDA.RadixSort. Every entry point
 * takes plain pointers and sizes (no C++ or torch types) and returns an rsort_status
 * (0 = ok) instead of the reference's print-and-exit CHECK (SourceCode/common/common.h:6-16);
 * include/radixsort.hpp restores the reference's exact C++ signatures and exit-on-error
 * behaviour on top of this ABI.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   rsort_u32            sortByDevice(h_in, n, h_out, numBits, blockSize)   Parallel7.cu:530-639
 *                        (host -> host, synchronous, device memory owned by the callee)
 *   rsort_u32_ex         the same plus the reference's per-phase timers       Parallel7.cu:532-538,633-638
 *   rsort_u32_device     the per-digit loop of sortByDevice on device buffers  Parallel7.cu:561-623
 *   rsort_pass_histogram histogram() + histogramKernel                        Parallel7.cu:318-359
 *   rsort_pass_scan      transpose() + scan() + transpose()                   Parallel7.cu:361-528, :596-598
 *   rsort_pass_scatter   sortLocallyDataBlocks() + scatter()                  Parallel7.cu:79-316, :568, :612
 *   rsort_pass_local_sort sortLocallyDataBlocks() alone                       Parallel7.cu:193-251
 *   rsort_u32_vendor     sortByThrust (the vendor comparator)                 Parallel7.cu:69-73
 *   (no counterpart)     rsort_u32_pairs*: key + u32 payload (BASELINE config 4)
 *   (no counterpart)     rsort_partition_device / rsort_bucket_starts: the multi-GPU
 *                        key-range partition step (BASELINE config 5)
 *
 * Semantics shared by every sort entry point:
 *   - keys are uint32_t, sorted ascending; k_bits in [1, 13] digit bits per pass (13: the reference's SMEM limit), passes at
 *     bit 0, k, 2k, ... < 32 (the last digit is short when k does not divide 32, exactly as
 *     Baseline1.cu:30-49);
 *   - output is bit-exact with Baseline1.cu's sortByHost; pairs are STABLE (equal keys keep
 *     their input order), i.e. equal to Baseline1's loop carrying the payload;
 *   - 0 <= n < 2^32; n == 0 is a no-op; `in` is never written; in == out is allowed;
 *   - device entry points are stream-ordered on `stream` (a hipStream_t, NULL = the null
 *     stream), do no allocation, no host synchronisation and are graph-capturable; they use
 *     the caller's workspace (rsort_workspace_size bytes, any alignment >= 256 B);
 *   - the device is the caller's current HIP device.
 */
#ifndef RSORT_H_
#define RSORT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(_WIN32)
#define RSORT_API
#else
#define RSORT_API __attribute__((visibility("default")))
#endif

typedef enum rsort_status {
    RSORT_OK = 0,
    RSORT_ERR_ARG = 1,        /* NULL pointer where data is required, bad option value */
    RSORT_ERR_BITS = 2,       /* k_bits outside [1, 13] */
    RSORT_ERR_SIZE = 3,       /* n < 0 or n >= 2^32 */
    RSORT_ERR_ALIGN = 4,      /* device buffer not 4-byte aligned */
    RSORT_ERR_ALLOC = 5,      /* hipMalloc / host allocation failed */
    RSORT_ERR_HIP = 6,        /* a HIP runtime call or kernel launch failed */
    RSORT_ERR_WORKSPACE = 7,  /* workspace too small */
    RSORT_ERR_NODEV = 8,      /* no HIP device visible */
    RSORT_ERR_CAPACITY = 9,   /* multi-GPU: this rank receives more keys than its output holds */
    RSORT_ERR_COMM = 10,      /* multi-GPU: an RCCL call failed */
    RSORT_ERR_CHECK = 11      /* host entries: an on-device self-check of the sort failed (rsort_plan_check) */
} rsort_status;

/* Local-rank algorithm inside a tile (all give the same, unique, stable result). */
typedef enum rsort_rank_algo {
    RSORT_RANK_MATCH = 0,  /* default: per-wave LDS digit counters; a key's rank is one
                              returning LDS add where the device serves same-address lanes in
                              lane order (probed once per device, rsort_lane_order_probe),
                              else the ballot peer-match below */
    RSORT_RANK_SPLIT = 1,  /* k successive block-local 1-bit splits, ballot/popcount scans
                              (the reference's algorithm, Parallel5.cu:79-159 / P7:79-191) */
    RSORT_RANK_BALLOT = 2  /* per-wave LDS digit counters + wave64 ballot peer-match */
} rsort_rank_algo;

/* Phases reported by the profiler (the reference's MEASURE_PORTION_EXECUTION_TIME buckets,
 * Parallel7.cu:634-637; the local sort is fused into the scatter kernel here). */
typedef enum rsort_phase {
    RSORT_PHASE_HISTOGRAM = 0,
    RSORT_PHASE_SCAN = 1,
    RSORT_PHASE_SCATTER = 2, /* fused block-local sort + rank + scatter: the measured pass */
    RSORT_PHASE_COPY = 3,    /* device-to-device copies (in-place sorts with an odd pass count) */
    RSORT_PHASE_PARTITION = 4, /* the multi-GPU key-range partition's scatter kernel (its histogram
                                  and scan count as HISTOGRAM and SCAN), kept apart from the sort's
                                  scatter passes so each has its own roofline figure */
    RSORT_PHASE_COUNT = 5
} rsort_phase;

typedef struct rsort_phase_times {
    double ms[RSORT_PHASE_COUNT];         /* summed kernel time per phase (hipEvent pairs) */
    int64_t launches[RSORT_PHASE_COUNT];  /* launches per phase */
    int64_t keys[RSORT_PHASE_COUNT];      /* keys processed per phase (sum over launches) */
} rsort_phase_times;

/* Geometry of one sort: tiles of tile_keys keys are locally sorted by one workgroup;
 * chunk_keys = tiles_per_chunk * tile_keys keys form one row of the chunk x digit table
 * (the reference's "block" of Baseline4.cu:79/Parallel7.cu:541, with the table stored
 * column-major [digit][chunk]). */
typedef struct rsort_plan {
    int64_t n;
    int32_t k_bits;
    int32_t passes;          /* ceil(32 / k_bits) */
    int32_t bins;            /* 2^k_bits */
    int32_t threads;         /* workgroup size */
    int32_t tile_keys;       /* keys per tile */
    int32_t pairs;           /* 1: key + value */
    int64_t tiles_per_chunk;
    int64_t chunk_keys;
    int64_t num_chunks;      /* workgroups per histogram / scatter launch */
    int64_t table_entries;   /* bins * num_chunks */
    int64_t scan_blocks;     /* workgroups of the table scan */
    size_t workspace_bytes;  /* for rsort_u32_device / rsort_u32_pairs_device */
} rsort_plan;

RSORT_API const char *rsort_status_string(int status);
RSORT_API int rsort_version(void); /* major * 10000 + minor * 100 + patch */

/* Geometry for (n, k_bits, pairs). tiles_per_chunk = 0 picks it from the current device's
 * CU count and the scatter kernel's occupancy (a fixed default when no device is visible). */
RSORT_API int rsort_plan_make(int64_t n, int k_bits, int pairs, int64_t tiles_per_chunk,
                              rsort_plan *plan);
/* Workspace bytes of a device sort: the ping-pong keys (4n, and 4n more for values), the chunk table and
 * scan sums (a few hundred KB), 256 B of check words, and by plan kind: k = 8 plans with 256 chunks (every
 * 2^23..2^31-key sort on a 256-CU MI355X) a FIXED ~65 MiB more -- the joint counts (256 KB), the cut plan
 * and its piece counts (~0.5 MB) and the per-chunk joint-count rows (256^3 words = 64 MiB + 256 KB), which
 * only skewed chunks write but every such plan reserves (near 2^23 keys that is more than the keys); k = 3,
 * 4 plans two more chunk tables. */
RSORT_API size_t rsort_workspace_size(int64_t n, int k_bits, int pairs);

/* ---------------------------------------------------------------- whole sort, device */
RSORT_API int rsort_u32_device(const uint32_t *d_in, uint32_t *d_out, int64_t n, int k_bits,
                               void *d_workspace, size_t workspace_bytes, void *stream);
RSORT_API int rsort_u32_pairs_device(const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                                     uint32_t *d_keys_out, uint32_t *d_vals_out, int64_t n,
                                     int k_bits, void *d_workspace, size_t workspace_bytes,
                                     void *stream);
/* Same, with an explicit plan (from rsort_plan_make) -- lets tests pin the geometry. */
RSORT_API int rsort_sort_planned(const rsort_plan *plan, const uint32_t *d_keys_in,
                                 const uint32_t *d_vals_in, uint32_t *d_keys_out,
                                 uint32_t *d_vals_out, void *d_workspace, size_t workspace_bytes,
                                 void *stream);

/* ---------------------------------------------------------------- whole sort, host -> host */
/* Synchronous drop-in for sortByDevice (Parallel7.cu:530): H2D, sort, D2H on the current
 * device with a library-owned, per-device cached workspace. */
RSORT_API int rsort_u32(const uint32_t *in, uint32_t *out, int64_t n, int k_bits);
/* Same; block_size is accepted for signature compatibility and has NO effect (the reference sets its
 * tile size from it, Parallel7.cu:541; here the gfx950 tile geometry follows k, n and pairs); `times`
 * (may be NULL) receives the per-phase kernel times of this call. */
RSORT_API int rsort_u32_ex(const uint32_t *in, uint32_t *out, int64_t n, int k_bits,
                           int block_size, rsort_phase_times *times);
RSORT_API int rsort_u32_pairs(const uint32_t *keys_in, const uint32_t *vals_in,
                              uint32_t *keys_out, uint32_t *vals_out, int64_t n, int k_bits);

/* ---------------------------------------------------------------- one digit pass, device */
/* digit(key) = (key >> shift) & (bins - 1). Table layout: d_table[digit * num_chunks + chunk]. */
RSORT_API int rsort_pass_histogram(const rsort_plan *plan, const uint32_t *d_keys, int shift,
                                   uint32_t *d_table, void *stream);
/* In-place exclusive scan of the column-major table; d_block_sums holds plan->scan_blocks
 * u32 of scratch. */
RSORT_API int rsort_pass_scan(const rsort_plan *plan, uint32_t *d_table, uint32_t *d_block_sums,
                              void *stream);
/* Fused block-local sort + global rank + scatter of one pass (vals may be NULL when
 * plan->pairs == 0). d_table is the scanned table of the same pass. */
RSORT_API int rsort_pass_scatter(const rsort_plan *plan, const uint32_t *d_keys_in,
                                 const uint32_t *d_vals_in, uint32_t *d_keys_out,
                                 uint32_t *d_vals_out, int shift, const uint32_t *d_table,
                                 void *stream);
/* Block-local stable sort of every tile by the digit, written in tile order (the state
 * sortLocallyDataBlocks leaves behind, Parallel7.cu:568). */
RSORT_API int rsort_pass_local_sort(const rsort_plan *plan, const uint32_t *d_keys_in,
                                    const uint32_t *d_vals_in, uint32_t *d_keys_out,
                                    uint32_t *d_vals_out, int shift, void *stream);

/* ---------------------------------------------------------------- options / profiling */
RSORT_API int rsort_set_rank_algo(int algo); /* rsort_rank_algo, process-wide */
RSORT_API int rsort_get_rank_algo(void);
/* Histograms carried between passes (default on), so passes read no keys for their histogram:
 *  - k = 8 plans with 256 chunks (digit-group chunks): every second pass takes the previous
 *    pass's digit groups as its chunks (the pass before counts (digit, next digit) pairs while
 *    it reads the keys); where the groups are unbalanced (skewed keys) it takes equal chunks
 *    and reads only the keys of the groups those chunks cut (all but each cut group's largest
 *    segment);
 *  - k = 3, 4 keys-only plans (next-digit counts): every pass adds the next pass's chunk table
 *    from where it writes each key; only pass 0 reads keys for a histogram.
 * Off: every pass counts its own histogram. Same output either way; process-wide. */
RSORT_API int rsort_set_group_chunks(int enable);
RSORT_API int rsort_get_group_chunks(void);
/* After a sort with `plan` and `d_workspace` has completed on `stream`: flags[i] says how odd
 * pass 2i+1 took its chunks (i < 2): 1 = the digit groups, 2 = equal chunks cutting unbalanced
 * groups (counted pieces), 0 = fixed chunks with a counted histogram (group chunks off, or plans
 * without them). Synchronises the stream. */
RSORT_API int rsort_group_flags(const rsort_plan *plan, const void *d_workspace, int *flags,
                                void *stream);
/* After a k = 8 digit-group sort with `plan` and `d_workspace` has completed on `stream`: how the cut plans
 * of passes 1 and 3 (rsort_group_flags 2) took the counts of their pieces, stats[4 * i + j] for pass 2i+1:
 * j = 0 key ranges counted from the keys, 1 row tasks (sums of the previous pass's per-chunk joint-count
 * rows), 2 direct adds (a chunk part whose keys all share one next digit), 3 key ranges counted negatively
 * (the complement of a piece inside a chunk). All 0 for a pass on whole groups or fixed chunks, and for
 * plans without digit groups. Synchronises the stream (tests and diagnostics). */
RSORT_API int rsort_cut_plan_stats(const rsort_plan *plan, const void *d_workspace, int *stats, void *stream);
/* After a sort with `plan` and `d_workspace` has completed on `stream`: *flags = 0 when every
 * on-device self-check of that sort passed; bit 0 (RSORT_CHECK_TABLE) = a k = 3, 4 pass found the
 * next-digit table it reads not holding n keys (the pass then wrote nothing; with RSORT_FEAT_TAIL_SCAN:
 * a tail scan found it so even after an acquire fence and a second sweep); bit 1 (RSORT_CHECK_RANK_ORDER)
 * = a lane-ordered scatter kernel's per-tile rank check failed: the device no longer served the lanes of
 * a returning LDS add in lane order (the premise of the default ranking, rsort_lane_order_probe), so
 * equal digits may have been written out of order -- in either case the sort's output is not
 * trustworthy. Every plan has the check words (256 B of the workspace); the rank check runs on the first
 * slot of every 8th full tile of each chunk (its first included), every pass. Synchronises the stream. The sort entry points are stream-ordered and do not
 * wait for the device, so they CANNOT return this check: they return RSORT_OK for such a sort, and
 * this call is the only way to learn of it. rsort_u32_device / rsort_u32_pairs_device use the plan
 * rsort_plan_make(n, k_bits, pairs, 0) gives, so pass that plan and the same workspace. The host
 * entries (rsort_u32, rsort_u32_ex, rsort_u32_pairs) wait for the device anyway: they read the check
 * themselves and return RSORT_ERR_CHECK for such a sort. Never observed failing. */
#define RSORT_CHECK_TABLE 1
#define RSORT_CHECK_RANK_ORDER 2
RSORT_API int rsort_plan_check(const rsort_plan *plan, const void *d_workspace, int *flags, void *stream);
/* Which carried-histogram scheme a sort with `plan` takes under the current process settings
 * (rsort_set_rank_algo, rsort_set_group_chunks), for outputs the whole-line kernels can write (any
 * 4-B-aligned keys output): a bitmask, or -RSORT_ERR_ARG for an invalid plan.
 *   RSORT_FEAT_GROUPS       k = 8, 256 chunks: digit-group chunks on the odd passes
 *   RSORT_FEAT_NEXT_DIGIT   k = 3, 4 keys: next-digit counts (only pass 0 reads keys for a histogram)
 *   RSORT_FEAT_RAW_TABLES   ... each pass after the first derives its starts from the raw counts in
 *                           every workgroup (plans of at most 1280 chunks: the per-workgroup sum
 *                           reads the whole R x C table)
 *   RSORT_FEAT_TAIL_SCAN    ... the last workgroup of each pass scans the next table instead (plans
 *                           with more chunks, e.g. a small tiles_per_chunk) */
#define RSORT_FEAT_GROUPS 1
#define RSORT_FEAT_NEXT_DIGIT 2
#define RSORT_FEAT_RAW_TABLES 4
#define RSORT_FEAT_TAIL_SCAN 8
RSORT_API int rsort_plan_features(const rsort_plan *plan);
/* TEST HOOK (never set in production): enable != 0 makes every raw-table sort (RSORT_FEAT_RAW_TABLES)
 * corrupt one word of the table pass 1 reads, as a lost update would; that pass's workgroups then
 * find the table not holding n keys, write nothing, and record it: rsort_plan_check reports bit 0 and
 * the host entries return RSORT_ERR_CHECK. Process-wide; returns the previous setting. */
RSORT_API int rsort_inject_table_fault(int enable);
/* TEST HOOK (never set in production): enable != 0 makes every lane-ordered scatter kernel swap the ranks
 * of the first two lanes of each digit in the slot its rank check looks at -- what a device serving
 * same-address LDS adds out of lane order would do. The sort is then unstable (wrong for keys, pairs out
 * of order), and the check catches it: rsort_plan_check reports bit 1 (RSORT_CHECK_RANK_ORDER), the host
 * entries return RSORT_ERR_CHECK. Process-wide; returns the previous setting. */
RSORT_API int rsort_inject_rank_fault(int enable);
/* The scatter kernel instantiations this library has launched since the last reset, ';'-joined
 * into buf (at most len - 1 characters and a NUL); returns the full length. reset != 0 clears the
 * record. A k = 8 digit-group sort launches a plain and a clustered-input kernel for each pass
 * after the first (the device picks one, the other leaves at once): both are listed. */
RSORT_API size_t rsort_scatter_kernels_used(char *buf, size_t len, int reset);
/* 1 if the current device's LDS returns same-address atomic adds in lane order (the default
 * ranking relies on it and falls back to ballots otherwise), 0 if not, < 0 on error. The
 * probe runs once per device (a few microseconds) and is cached. */
RSORT_API int rsort_lane_order_probe(void);
/* Between begin and end, every launch made by this library records hipEvents around its
 * phases; end synchronises those events and returns the per-phase sums. */
RSORT_API int rsort_profile_begin(void);
RSORT_API int rsort_profile_end(rsort_phase_times *out);

/* ---------------------------------------------------------------- multi-GPU building blocks */
/* Stable partition of n keys (and values) into num_buckets (<= 32) key ranges:
 * bucket(key) = #{i : key >= splitters[i]} for the num_buckets-1 ascending host-side
 * splitters. Output is bucket-major and stable; d_bucket_starts[num_buckets + 1] receives
 * the exclusive bucket offsets (last = n). Workspace: rsort_partition_workspace_size. */
RSORT_API size_t rsort_partition_workspace_size(int64_t n, int num_buckets, int pairs);
RSORT_API int rsort_partition_device(const uint32_t *d_keys_in, const uint32_t *d_vals_in,
                                     uint32_t *d_keys_out, uint32_t *d_vals_out, int64_t n,
                                     const uint32_t *splitters, int num_buckets,
                                     uint32_t *d_bucket_starts, void *d_workspace,
                                     size_t workspace_bytes, void *stream);
/* After rsort_partition_device(n, num_buckets, pairs) has completed on `stream` in `d_workspace`: its
 * on-device self-check, as rsort_plan_check reports a sort's (bit 1: its scatter's rank check failed).
 * Synchronises the stream. rsort_u32_multi* reads it after every partition and returns RSORT_ERR_CHECK
 * on every rank when any rank's failed. */
RSORT_API int rsort_partition_check(int64_t n, int num_buckets, int pairs, const void *d_workspace, int *flags,
                                    void *stream);
/* Histogram of the top `top_bits` (1..12) bits of n keys into d_hist[2^top_bits] (u32,
 * overwritten). Workspace: rsort_workspace_size(n, top_bits, 0). */
RSORT_API int rsort_top_histogram(const uint32_t *d_keys, int64_t n, int top_bits,
                                  uint32_t *d_hist, void *d_workspace, size_t workspace_bytes,
                                  void *stream);
/* The same histogram over a sample: the keys of every `stride`-th block of 256 (block b is
 * counted iff b % stride == 0; stride 1 = every key). No workspace. The multi-GPU sort chooses
 * its splitters from this (stride 16: a sixteenth of the keys read). */
RSORT_API int rsort_top_histogram_sampled(const uint32_t *d_keys, int64_t n, int top_bits,
                                          int stride, uint32_t *d_hist, void *stream);

/* ---------------------------------------------------------------- multi-GPU planning (host only) */
/* The host-side decisions of the multi-GPU sort, as pure functions (no device, no communicator):
 * rsort_u32_multi* and cuda.radixsort_amd/multi.py both call them, and tests drive them on the
 * CPU at any world size. Every rank calls them with the same gathered inputs and gets the same
 * answer, so the ranks agree on every decision (including errors) without another collective.
 *
 * 1. Sampling. Given every rank's key count, the sampling stride (the same on every rank) and
 *    each rank's sample count: rank r samples key[min(n_r - 1, j * stride + stride / 2)] for
 *    j < count[r] and pads its row to row_len with 0xFFFFFFFF. Every sample then stands for
 *    `stride` keys, so the sorted union of the rows gives the global quantiles directly: the
 *    i-th of world - 1 splitters is sorted[floor(i * total_samples / world)]. */
#define RSORT_MAX_RANKS 16
typedef struct rsort_sample_plan {
    int32_t world;
    int64_t stride;                  /* keys per sample, >= 1 */
    int64_t count[RSORT_MAX_RANKS];  /* samples taken by each rank */
    int64_t row_len;                 /* samples per rank in the gathered buffer (max count, >= 1) */
    int64_t total;                   /* sum of count */
} rsort_sample_plan;
RSORT_API int rsort_multi_sample_plan(int world, const int64_t *n_per_rank, int64_t samples_per_rank,
                                      rsort_sample_plan *out);
/* The device side of step 1: d_out[j] = d_keys[min(n - 1, j * stride + stride / 2)] for j < count,
 * 0xFFFFFFFF for count <= j < row_len. */
RSORT_API int rsort_sample_device(const uint32_t *d_keys, int64_t n, int64_t stride, int64_t count,
                                  int64_t row_len, uint32_t *d_out, void *stream);
/* Index into the sorted gathered samples of splitter i (1 <= i < world). */
RSORT_API int64_t rsort_multi_quantile_index(const rsort_sample_plan *sp, int i);

/* 2. Splitters. From the world - 1 quantile keys v_1 <= ... <= v_{world-1}: the partition's
 * splitters and, for each rank boundary, where it cuts. Every distinct v gets a bucket of its own,
 * [v, v + 1) ("equal keys"), between the buckets of the keys below and above it, and boundary r
 * cuts INSIDE the equal-keys bucket of v_r at the position that balances the ranks: a run of equal
 * keys (a hot key, duplicate-heavy input) is split across ranks in global (source rank, position)
 * order, which keeps the sort stable. (2 * (world - 1) <= 30 splitters: within the partition's 32
 * buckets at every world size.) */
typedef struct rsort_multi_splitters {
    int32_t world;
    int32_t nsplit;                                 /* partition splitters (buckets = nsplit + 1) */
    uint32_t split[2 * (RSORT_MAX_RANKS - 1)];      /* non-decreasing */
    int32_t cut_bucket[RSORT_MAX_RANKS];            /* boundary r (1..world-1) lies in this bucket */
    int32_t cut_inside[RSORT_MAX_RANKS];            /* 1: anywhere inside it (equal keys); 0: at its start */
} rsort_multi_splitters;
RSORT_API int rsort_multi_splitters_make(int world, const uint32_t *quantile_keys, rsort_multi_splitters *out);
/* The same with a hot flag per quantile key (hot[r - 1] for boundary r; nullptr: every key hot, which is
 * rsort_multi_splitters_make). Only a hot key -- one whose run in the sorted sample is long enough that
 * sending all its copies to one rank would unbalance the ranks -- gets its equal-keys bucket; the others
 * are plain splitters (boundary r at the start of v_r's bucket: all copies of v_r go to rank r), one
 * bucket fewer each. Equal consecutive quantile keys are always one hot run. rsort_u32_multi* flags a key
 * hot when the sample holds it `world * 128`-th of the samples away on either side (a run of >= ~1/64 of
 * a rank's share): distinct keys get world - 1 splitters instead of 2 (world - 1). */
RSORT_API int rsort_multi_splitters_make_hot(int world, const uint32_t *quantile_keys, const int *hot,
                                             rsort_multi_splitters *out);

/* 3. Exchange. counts[s * buckets + b] = keys of rank s's partition in bucket b (the row every
 * rank gathers after partitioning); capacity[r] = output room of rank r. For rank `me`: what it
 * sends to each rank (offset and count in its partitioned buffer), what it receives from each
 * rank (in source-rank order: offset and count in its output), its output count and global
 * offset. RSORT_ERR_CAPACITY (with over_capacity = the first rank concerned) when ANY rank would
 * receive more than its capacity -- every rank sees the same matrix, so all ranks return it
 * together, before any key moves. */
typedef struct rsort_exchange_plan {
    int32_t world, me;
    int64_t send_off[RSORT_MAX_RANKS], send_cnt[RSORT_MAX_RANKS];
    int64_t recv_off[RSORT_MAX_RANKS], recv_cnt[RSORT_MAX_RANKS];
    int64_t n_recv;        /* keys this rank ends with */
    int64_t offset;        /* global rank of its first key */
    int64_t total;         /* keys over all ranks */
    int64_t max_message;   /* largest message between two different ranks, anywhere (keys) */
    int32_t over_capacity; /* -1, or the lowest rank whose output would overflow */
} rsort_exchange_plan;
RSORT_API int rsort_multi_exchange_plan(int world, int me, int buckets, const int64_t *counts,
                                        const rsort_multi_splitters *sp, const int64_t *capacity,
                                        rsort_exchange_plan *out);

/* 4. Exchange rounds. Messages of up to max_message keys (the plan's max_message), at most `limit`
 * keys each: *rounds equal pieces of *piece keys, a multiple of 64 keys (rounded up where that stays
 * within the limit -- a message under the limit is one round -- else down: never above the limit;
 * >= 64), rounds * piece >= max_message. (0, 0) for max_message 0. */
RSORT_API int rsort_multi_exchange_rounds(int64_t max_message, int64_t limit, int64_t *rounds, int64_t *piece);

/* ---------------------------------------------------------------- multi-GPU sort */
/* One rank per GPU (the reference is single-GPU, Parallel7.cu:10). Every rank
 * passes its n local keys (and values); on return rank r's d_keys_out[0 .. *out_n) holds the keys
 * of global ranks [*out_offset, *out_offset + *out_n) of the sorted union, i.e. concatenating the
 * ranks' outputs in rank order gives Baseline1's result; pairs stay stable (equal keys keep their
 * (source rank, position) order). Steps: all-gather of the key counts -> a regular sample of the
 * keys, all-gathered and sorted on the device -> world - 1 quantile keys -> splitters with a
 * bucket of its own for each hot quantile key, so a run of equal keys is split across
 * ranks -> stable partition -> all-gather of the bucket counts and capacities -> the exchange
 * plan (the same on every rank) -> one exchange (own range by a device copy, the rest point to
 * point in rounds of <= 2^28 keys per message) -> local LSD sort. Synchronises `stream` four
 * times (counts are needed on the host).
 * capacity: room in d_keys_out / d_vals_out. RSORT_ERR_CAPACITY when ANY rank would receive more
 * than its capacity: every rank returns it, before any key moves (balanced output needs about
 * total / world plus the sampling error, ~0.1 %). Up to RSORT_MAX_RANKS ranks.
 * Errors: a failure on one rank before the exchange (bad k_bits / sizes / pointers, a workspace
 * too small, a device error in sampling, sample sort or partition) travels in a status word of the
 * next all-gather, and EVERY rank returns the lowest rank's status together -- no rank is left
 * waiting in a collective (a rank that dies instead is caught by the RCCL timeout below). Only a transport that cannot run at all (NULL
 * transport or workspace, a workspace smaller than the collectives' control buffers) returns at
 * once on that rank. Failures in or after the exchange (the exchange itself, the local sort) are
 * the failing rank's own. */
RSORT_API size_t rsort_multi_workspace_size(int64_t n, int64_t capacity, int k_bits, int pairs, int world);
/* Over an RCCL communicator (`nccl_comm` is an ncclComm_t; RCCL result codes are all checked,
 * RSORT_ERR_COMM on failure). Every RCCL call is bounded: the sort waits for each collective and
 * exchange round to complete (host-polled), and when one has not completed within the communicator
 * timeout (rsort_set_comm_timeout) -- a peer that died or never joined -- or RCCL reports an
 * asynchronous error, it aborts the communicator (ncclCommAbort) and returns RSORT_ERR_COMM. The
 * communicator is then gone: do not use or destroy it again (rsort_rccl_comm_destroy knows it). */
RSORT_API int rsort_u32_multi(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n,
                              uint32_t *d_keys_out, uint32_t *d_vals_out, int64_t capacity,
                              int64_t *out_n, int64_t *out_offset, int k_bits, void *nccl_comm,
                              void *d_workspace, size_t workspace_bytes, void *stream);

/* RCCL communicators with bounded setup (replaces ncclGetUniqueId / ncclCommInitRank for the
 * callers of rsort_u32_multi): the id (NCCL_UNIQUE_ID_BYTES = 128 bytes) is made on one rank and
 * sent to the others out of band; init creates the rank's communicator on the current device,
 * non-blocking (ncclCommInitRankConfig, blocking = 0), and polls it until it is ready -- or, after
 * timeout_ms (<= 0: the rsort_set_comm_timeout value), aborts it and returns RSORT_ERR_COMM, so a
 * peer that never joins cannot hang this rank. destroy: ncclCommDestroy, or nothing for a
 * communicator a timeout already aborted. */
RSORT_API int rsort_rccl_unique_id(void *id128);
RSORT_API int rsort_rccl_comm_init(void **comm, int world, int rank, const void *id128, int timeout_ms);
RSORT_API int rsort_rccl_comm_destroy(void *comm);
/* How long one RCCL step of rsort_u32_multi (a collective, an exchange round, the communicator's
 * setup) may take before the communicator is aborted: default 300000 ms. Process-wide; returns the
 * previous value; values <= 0 leave it unchanged. */
RSORT_API int rsort_set_comm_timeout(int timeout_ms);

/* Options of rsort_u32_multi* (process-wide; returns the previous flags):
 *  RSORT_MULTI_OVERLAP  every rank's key range is cut in two at a sampled quantile (the planning
 *                       functions run for 2 x world ranks, world <= 8): the lower halves are
 *                       exchanged first, and each rank sorts its lower half on a second stream
 *                       while the upper halves are exchanged; same output.
 *  RSORT_MULTI_NO_OVERLAP  never cut the ranges in two.
 *  Neither: the overlap runs for 2 <= world <= 8 (RSORT_MULTI_AUTO_OVERLAP_MAX_WORLD; 2 x world <=
 *                       RSORT_MAX_RANKS virtual ranks), where it is predicted faster at every size
 *                       (components measured on one GPU; at world 8 the partition into
 *                       16 buckets costs 2.49 ms, as the 8 buckets without halves).
 *  RSORT_MULTI_FULL     run the whole protocol also at world 1 (sample, partition into one
 *                       bucket, self exchange): for tests and overhead measurements. By default
 *                       one rank sorts its keys directly (the partition would be a copy). */
#define RSORT_MULTI_OVERLAP 1
#define RSORT_MULTI_FULL 2
#define RSORT_MULTI_NO_OVERLAP 4
#define RSORT_MULTI_AUTO_OVERLAP_MAX_WORLD 8
RSORT_API int rsort_set_multi_options(int flags);

/* Per-phase record of a multi-GPU sort (rsort_u32_multi*), for the N-GPU bench line. Off by
 * default; while on, every multi-GPU sort records hipEvents on its stream at the phase boundaries
 * and synchronises its stream before returning (so it is no longer asynchronous), and the calling
 * thread's last sort is kept for rsort_multi_last_stats. Phases on the caller's stream:
 *   plan       count all-gather, sampling, sample all-gather + device sort, splitters
 *   partition  the stable partition, the count/capacity all-gather, the exchange plan
 *   exchange   every exchange round (and the own range's device copy beside it)
 *   local_sort the LSD sort of what arrived
 * With RSORT_MULTI_OVERLAP the lower half's sort runs on a second stream during the upper half's
 * exchange: `exchange` then ends when the last message has arrived and `local_sort` is the rest. */
typedef struct rsort_multi_stats {
    int32_t world;       /* ranks of the communicator (rsort_u32_multi: ncclCommCount) */
    int32_t rank;        /* this rank (rsort_u32_multi: ncclCommUserRank) */
    int32_t halves;      /* 1, or 2 when the overlap ran (RSORT_MULTI_OVERLAP, or its automatic use) */
    int32_t direct;      /* 1: world 1 without RSORT_MULTI_FULL, sorted directly (phases: local_sort) */
    int64_t rounds;      /* exchange rounds (messages per peer and array) */
    int64_t bytes_per_key; /* 4 (keys) or 8 (key + value) */
    int64_t send_keys[RSORT_MAX_RANKS]; /* keys this rank sent to each rank (own entry: the device copy) */
    int64_t recv_keys[RSORT_MAX_RANKS]; /* keys it received from each rank */
    int64_t n_in, n_out; /* keys in, keys out on this rank */
    double ms_plan, ms_partition, ms_exchange, ms_local_sort, ms_total;
} rsort_multi_stats;
RSORT_API int rsort_multi_set_profiling(int enable); /* process-wide; returns the previous setting */
/* The calling thread's last multi-GPU sort made while profiling was on (RSORT_ERR_ARG if none). */
RSORT_API int rsort_multi_last_stats(rsort_multi_stats *out);

/* TEST HOOK (fault injection for the error-agreement tests; never set in production): the next
 * multi-GPU sorts of rank `rank` fail with `status` at `stage` (1: the sample sort, after the sample
 * all-gather; 2: the partition), as a device failure there would. rank < 0 clears the hook. */
RSORT_API int rsort_multi_inject_failure(int rank, int stage, int status);

/* Largest message of one exchange round, in keys (default and maximum 2^28 = 1 GiB; >= 64).
 * Messages are cut into equal pieces of a multiple of 64 keys, never above the limit, even when it
 * is not a multiple of 64 (rsort_multi_exchange_rounds). Process-wide; returns the previous value. Tests
 * set small values to force several rounds. */
RSORT_API int64_t rsort_set_exchange_piece(int64_t keys);

/* The communication the multi-GPU sort needs, as a plug-in (RCCL is one implementation, the
 * in-process loopback below another; MPI or a host transport could be a third). Both calls are
 * made by every rank in the same order; they return 0 or a nonzero rsort_status. */
typedef struct rsort_transport {
    void *ctx;
    int32_t world, rank;
    /* every rank contributes `bytes` device bytes at d_send; d_recv (world * bytes) receives the
     * contributions in rank order. Stream-ordered on `stream` (or synchronous). */
    int (*allgather)(void *ctx, const void *d_send, void *d_recv, size_t bytes, void *stream);
    /* one round of messages: for each peer p != rank, send send_bytes[p] bytes from d_send[p] and
     * receive recv_bytes[p] bytes into d_recv[p] (0 = none; entry `rank` is always 0). */
    int (*exchange)(void *ctx, void *const *d_send, const size_t *send_bytes, void *const *d_recv,
                    const size_t *recv_bytes, void *stream);
} rsort_transport;
RSORT_API int rsort_u32_multi_transport(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n,
                                        uint32_t *d_keys_out, uint32_t *d_vals_out, int64_t capacity,
                                        int64_t *out_n, int64_t *out_offset, int k_bits,
                                        const rsort_transport *transport, void *d_workspace,
                                        size_t workspace_bytes, void *stream);
/* A transport over HOST memory (MPI, gloo, sockets, ...), wrapped into an rsort_transport: the
 * wrapper synchronises the stream, stages the device bytes through host buffers it owns, calls
 * the host functions (same contract as rsort_transport, host pointers) and copies the results back
 * to the device. bench.py's N-rank rehearsal on one card and the gloo tests run the C protocol this
 * way; the product path on a multi-GPU node is RCCL (rsort_u32_multi). The wrapper keeps a copy of
 * *host; free it with rsort_host_transport_free after the last sort. */
typedef struct rsort_host_transport {
    void *ctx;
    int32_t world, rank;
    int (*allgather)(void *ctx, const void *h_send, void *h_recv, size_t bytes);
    int (*exchange)(void *ctx, void *const *h_send, const size_t *send_bytes, void *const *h_recv,
                    const size_t *recv_bytes);
} rsort_host_transport;
RSORT_API int rsort_host_transport_wrap(const rsort_host_transport *host, rsort_transport *out);
RSORT_API void rsort_host_transport_free(rsort_transport *wrapped);

/* In-process loopback world: `world` ranks, one host thread each, calling
 * rsort_u32_multi_transport concurrently on their own streams (one device, or devices with peer
 * access). Collectives are a host rendezvous plus device-to-device copies; a rank that waits more
 * than 120 s fails with RSORT_ERR_COMM (and so do the others). For testing the multi-GPU path on
 * one GPU (RCCL refuses two ranks on one device). */
RSORT_API int rsort_loopback_create(int world, void **group);
RSORT_API int rsort_loopback_transport(void *group, int rank, rsort_transport *out);
RSORT_API void rsort_loopback_destroy(void *group);

/* ---------------------------------------------------------------- vendor comparator */
/* rocPRIM's device radix sort (what sortByThrust resolves to on ROCm), for the
 * "vendor ceiling" column. */
RSORT_API size_t rsort_vendor_workspace_size(int64_t n);
RSORT_API int rsort_u32_vendor_device(const uint32_t *d_in, uint32_t *d_out, int64_t n,
                                      void *d_workspace, size_t workspace_bytes, void *stream);
RSORT_API int rsort_u32_vendor(const uint32_t *in, uint32_t *out, int64_t n);

/* ---------------------------------------------------------------- output check */
/* d_out[0] = sum over i of fmix64(d_vals[i] << 32 | d_keys[i]) mod 2^64 (d_vals may be NULL: 0),
 * an order-independent fingerprint of the (key, value) multiset; d_out[1] = #{i : d_keys[i] >
 * d_keys[i + 1]}. A correct sort keeps d_out[0] and has d_out[1] == 0 (bench.py checks its timed
 * output this way; the parity tests compare with the oracle instead). d_out: 2 u64, device. */
RSORT_API int rsort_fingerprint_device(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n,
                                       uint64_t *d_out, void *stream);

/* ---------------------------------------------------------------- synthetic workloads */
/* key[i] = high 32 bits of splitmix64(seed + i). */
RSORT_API int rsort_gen_uniform(uint32_t *d_out, int64_t n, uint64_t seed, void *stream);
/* key[i] = fmix32(rank), rank = lower_bound(d_cdf[0..ranks), u_i) with u_i the uniform
 * stream above; d_cdf is the inclusive Zipf CDF scaled to u32 (last entry 2^32-1). */
RSORT_API int rsort_gen_zipf(uint32_t *d_out, int64_t n, uint64_t seed, const uint32_t *d_cdf,
                             int64_t ranks, void *stream);
/* d_out[i] = base + i */
RSORT_API int rsort_gen_iota(uint32_t *d_out, int64_t n, uint32_t base, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RSORT_H_ */
