// rsort_exchange.cpp -- the host-side decisions of the multi-GPU sort as pure functions (no HIP,
// no communicator): sampling plan, splitters with equal-key buckets for hot keys, and the exchange plan with
// its capacity check (include/rsort.h, "multi-GPU planning").
//
// No reference counterpart (the reference sorts on one GPU, Parallel7.cu:10/:697); SURVEY.md §8e
// / BASELINE config 5. rsort_u32_multi* (rsort_multi.cpp) and multi.py call these with the same
// gathered inputs on every rank, so every rank reaches the same decision -- including an error --
// without another collective. Compiled into librsort.so and, for tests/test_exchange.py, into a
// CPU-only executable under -fsanitize=address,undefined (this file includes nothing from HIP).
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "rsort.h"

namespace {

constexpr int kMaxRanks = RSORT_MAX_RANKS;
// every world: 2 * (world - 1) <= 30 splitters, within the partition's 31 (32 buckets)

}  // namespace

extern "C" {

int rsort_multi_sample_plan(int world, const int64_t *n_per_rank, int64_t samples_per_rank, rsort_sample_plan *out) {
    if (!out || !n_per_rank || world < 1 || world > kMaxRanks || samples_per_rank < 1) return RSORT_ERR_ARG;
    memset(out, 0, sizeof(*out));
    int64_t total_keys = 0;
    for (int r = 0; r < world; ++r) {
        if (n_per_rank[r] < 0 || n_per_rank[r] >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
        total_keys += n_per_rank[r];
    }
    // one stride for every rank: each sample stands for the same number of keys
    const int64_t budget = samples_per_rank * world;
    int64_t stride = total_keys > 0 ? (total_keys + budget - 1) / budget : 1;
    if (stride < 1) stride = 1;
    out->world = world;
    out->stride = stride;
    int64_t row = 1;
    for (int r = 0; r < world; ++r) {
        out->count[r] = (n_per_rank[r] + stride - 1) / stride;
        out->total += out->count[r];
        row = std::max(row, out->count[r]);
    }
    out->row_len = row;
    return RSORT_OK;
}

int64_t rsort_multi_quantile_index(const rsort_sample_plan *sp, int i) {
    if (!sp || i < 1 || i >= sp->world || sp->total <= 0) return 0;
    int64_t q = (int64_t)(((__int128)i * sp->total) / sp->world);
    return q < sp->total ? q : sp->total - 1;
}

int rsort_multi_splitters_make(int world, const uint32_t *quantile_keys, rsort_multi_splitters *out) {
    return rsort_multi_splitters_make_hot(world, quantile_keys, nullptr, out);
}

int rsort_multi_splitters_make_hot(int world, const uint32_t *quantile_keys, const int *hot,
                                   rsort_multi_splitters *out) {
    if (!out || world < 1 || world > kMaxRanks || (world > 1 && !quantile_keys)) return RSORT_ERR_ARG;
    memset(out, 0, sizeof(*out));
    out->world = world;
    for (int i = 1; i + 1 < world; ++i)
        if (quantile_keys[i] < quantile_keys[i - 1]) return RSORT_ERR_ARG;
    // A hot quantile key v (hot == nullptr: every one) gets its own bucket [v, v + 1) between the
    // buckets below and above it, and the rank boundary cuts INSIDE it at the balancing position: a
    // run of equal keys is split across ranks. A key that is not hot is a plain splitter: the ranks
    // meet at v (its few copies all go up), one bucket fewer -- for distinct keys every quantile is
    // plain, and the partition computes a digit from world - 1 splitters instead of 2 (world - 1)
    // (2^30 keys into 8 ranks: 2.44 ms against 2.64 ms with 15 buckets, dev/part_lab.py). Equal
    // consecutive quantile keys are one run: one bucket, hot.
    // bucket j >= 1 is [split[j - 1], split[j]); the bucket starting at split[i] is bucket i + 1
    int r = 1;
    while (r < world) {
        const uint32_t v = quantile_keys[r - 1];
        int e = r + 1;  // boundaries r .. e - 1 share the key v
        while (e < world && quantile_keys[e - 1] == v) ++e;
        bool eq = hot == nullptr || e - r > 1;
        for (int b = r; b < e && !eq; ++b) eq = hot[b - 1] != 0;
        const int at = out->nsplit;
        out->split[out->nsplit++] = v;
        // key 0xFFFFFFFF: its bucket [v, v + 1) is everything from v on (no upper splitter, and the
        // bucket above it does not exist)
        if (eq && v != 0xFFFFFFFFu) out->split[out->nsplit++] = v + 1u;
        for (int b = r; b < e; ++b) {
            out->cut_bucket[b] = at + 1;
            out->cut_inside[b] = eq ? 1 : 0;
        }
        r = e;
    }
    return RSORT_OK;
}

int rsort_multi_exchange_plan(int world, int me, int buckets, const int64_t *counts, const rsort_multi_splitters *sp,
                              const int64_t *capacity, rsort_exchange_plan *out) {
    if (!out || !counts || !sp || !capacity) return RSORT_ERR_ARG;
    if (world < 1 || world > kMaxRanks || me < 0 || me >= world || sp->world != world) return RSORT_ERR_ARG;
    if (buckets != sp->nsplit + 1 || buckets < 1 || buckets > 2 * kMaxRanks) return RSORT_ERR_ARG;
    memset(out, 0, sizeof(*out));
    out->world = world;
    out->me = me;
    out->over_capacity = -1;
    for (int i = 0; i < world * buckets; ++i)
        if (counts[i] < 0) return RSORT_ERR_ARG;
    for (int r = 1; r < world; ++r)
        if (sp->cut_bucket[r] < 0 || sp->cut_bucket[r] >= buckets ||
            (r > 1 && sp->cut_bucket[r] < sp->cut_bucket[r - 1]))
            return RSORT_ERR_ARG;

    // global bucket starts and each source's local bucket starts
    int64_t gb[2 * kMaxRanks + 1];
    int64_t lb[kMaxRanks][2 * kMaxRanks + 1];
    gb[0] = 0;
    for (int b = 0; b < buckets; ++b) {
        int64_t t = 0;
        for (int s = 0; s < world; ++s) t += counts[s * buckets + b];
        gb[b + 1] = gb[b] + t;
    }
    for (int s = 0; s < world; ++s) {
        lb[s][0] = 0;
        for (int b = 0; b < buckets; ++b) lb[s][b + 1] = lb[s][b] + counts[s * buckets + b];
    }
    const int64_t total = gb[buckets];
    out->total = total;

    // boundary r: global position G[r] of the first key of rank r, and cut[s][r] = the first key of
    // source s's partition that goes to rank r or above
    int64_t G[kMaxRanks + 1];
    int64_t cut[kMaxRanks][kMaxRanks + 1];
    G[0] = 0;
    G[world] = total;
    for (int s = 0; s < world; ++s) {
        cut[s][0] = 0;
        cut[s][world] = lb[s][buckets];
    }
    for (int r = 1; r < world; ++r) {
        const int b = sp->cut_bucket[r];
        if (sp->cut_inside[r]) {
            // inside the bucket of equal keys: balance the ranks (target r * total / world), the
            // bucket's keys ordered by (source rank, position), which is their stable order
            const int64_t target = (int64_t)(((__int128)r * total) / world);
            int64_t g = std::min(std::max(target, gb[b]), gb[b + 1]);
            g = std::max(g, G[r - 1]);
            G[r] = g;
            int64_t before = gb[b];
            for (int s = 0; s < world; ++s) {
                const int64_t c = counts[s * buckets + b];
                const int64_t q = std::min(std::max(g - before, (int64_t)0), c);
                cut[s][r] = lb[s][b] + q;
                before += c;
            }
        } else {
            G[r] = std::max(gb[b], G[r - 1]);
            for (int s = 0; s < world; ++s) cut[s][r] = lb[s][b];
        }
    }
    // monotone cuts (guaranteed by the above; checked so a bad input cannot yield negative counts)
    for (int s = 0; s < world; ++s)
        for (int r = 1; r <= world; ++r)
            if (cut[s][r] < cut[s][r - 1]) return RSORT_ERR_ARG;

    int64_t biggest = 0;
    for (int r = 0; r < world; ++r) {
        int64_t nr = 0;
        for (int s = 0; s < world; ++s) {
            const int64_t m = cut[s][r + 1] - cut[s][r];
            nr += m;
            if (s != r) biggest = std::max(biggest, m);
        }
        if (nr > capacity[r] && out->over_capacity < 0) out->over_capacity = r;
    }
    out->max_message = biggest;
    int64_t ro = 0;
    for (int s = 0; s < world; ++s) {
        out->send_off[s] = cut[me][s];
        out->send_cnt[s] = cut[me][s + 1] - cut[me][s];
        out->recv_off[s] = ro;
        out->recv_cnt[s] = cut[s][me + 1] - cut[s][me];
        ro += out->recv_cnt[s];
    }
    out->n_recv = ro;
    out->offset = G[me];
    return out->over_capacity >= 0 ? RSORT_ERR_CAPACITY : RSORT_OK;
}

int rsort_multi_exchange_rounds(int64_t max_message, int64_t limit, int64_t *rounds, int64_t *piece) {
    if (!rounds || !piece || max_message < 0 || limit < 1) return RSORT_ERR_ARG;
    *rounds = 0;
    *piece = 0;
    if (max_message == 0) return RSORT_OK;
    limit = std::max<int64_t>(limit, 64);
    const int64_t r0 = (max_message + limit - 1) / limit;  // rounds at the limit
    int64_t p = (max_message + r0 - 1) / r0;               // equal pieces, <= limit
    // a multiple of 64: rounded up where that stays within the limit (r0 rounds; rounding down made a
    // one-round message of 2^27 + 6 keys take a second round of 6 keys), else down (never above it)
    const int64_t up = (p + 63) / 64 * 64;
    p = up <= limit ? up : std::max<int64_t>(64, p / 64 * 64);
    *piece = p;
    *rounds = (max_message + p - 1) / p;
    return RSORT_OK;
}

}  // extern "C"
