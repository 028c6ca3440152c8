// exchange_fuzz.cpp -- CPU-only driver for the multi-GPU planning functions
// (cuda.radixsort_amd/csrc/rsort_exchange.cpp), built with -fsanitize=address,undefined by
// tests/test_exchange.py. Random worlds 1..16, ragged / empty / skewed bucket counts, equal-key
// and bucket-edge cuts, tight capacities; checks the invariants every rank relies on:
//   * each rank's sends cover its partition exactly, in order; receives are in source order;
//   * what rank s sends to r is what r expects from s (the plans of all ranks agree);
//   * output counts sum to the total, offsets are their exclusive scan;
//   * the capacity verdict is the same on every rank;
//   * cuts inside an equal-keys bucket land where the balanced target says, clamped to it.
// Prints "ok <cases>" and exits 0, or the first violation and exits 1.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "rsort.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

#define FAIL(...)                         \
    do {                                  \
        printf("case %d: ", c);           \
        printf(__VA_ARGS__);              \
        printf("\n");                     \
        return 1;                         \
    } while (0)

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 20000;
    // exchange rounds: pieces never above the limit, a multiple of 64, covering the message
    for (int c = 0; c < cases; ++c) {
        const int64_t m = (int64_t)(next() % ((uint64_t)1 << (next() % 41)));
        const int64_t limit = 1 + (int64_t)(next() % ((uint64_t)1 << (1 + next() % 30)));
        int64_t r = -1, p = -1;
        if (rsort_multi_exchange_rounds(m, limit, &r, &p) != RSORT_OK) FAIL("exchange_rounds failed");
        if (m == 0 && (r != 0 || p != 0)) FAIL("rounds of an empty message");
        if (m > 0 && (p < 64 || p % 64 != 0 || p > std::max<int64_t>(limit, 64) || r * p < m || (r - 1) * p >= m))
            FAIL("rounds m=%lld limit=%lld -> %lld x %lld", (long long)m, (long long)limit, (long long)r, (long long)p);
    }
    for (int c = 0; c < cases; ++c) {
        const int world = 1 + (int)(next() % RSORT_MAX_RANKS);
        // quantile keys: sorted, with repeats and the extreme keys
        std::vector<uint32_t> q(world > 1 ? world - 1 : 1);
        const int mode = (int)(next() % 4);
        for (auto &x : q) {
            x = (uint32_t)next();
            if (mode == 1) x &= 0xFu;                 // many repeats
            if (mode == 2) x = (next() & 1) ? 0xFFFFFFFFu : 0u;
            if (mode == 3) x = 0xC0FFEEu;             // all equal
        }
        std::sort(q.begin(), q.end());
        rsort_multi_splitters sp;
        // every key hot (rsort_multi_splitters_make) or random hot flags (make_hot)
        std::vector<int> hot(q.size());
        for (auto &h : hot) h = (int)(next() & 1);
        if ((next() & 1) ? rsort_multi_splitters_make(world, q.data(), &sp) != RSORT_OK
                         : rsort_multi_splitters_make_hot(world, q.data(), hot.data(), &sp) != RSORT_OK)
            FAIL("splitters_make failed");
        for (int i = 1; i < sp.nsplit; ++i)
            if (sp.split[i] < sp.split[i - 1]) FAIL("splitters not monotone");
        const int buckets = sp.nsplit + 1;
        if (buckets > 32) FAIL("more than 32 buckets (%d)", buckets);
        // bucket counts per source rank
        std::vector<int64_t> counts((size_t)world * buckets), n(world, 0);
        const int cmode = (int)(next() % 4);
        for (int s = 0; s < world; ++s)
            for (int b = 0; b < buckets; ++b) {
                int64_t v = (int64_t)(next() % 1000);
                if (cmode == 1 && (next() % 3)) v = 0;                      // sparse / empty ranks
                if (cmode == 2 && (b % 2 == 1)) v *= 1000;                 // hot equal-key buckets
                if (cmode == 3) v = (int64_t)(next() % 3);
                counts[(size_t)s * buckets + b] = v;
                n[s] += v;
            }
        int64_t total = 0;
        for (int s = 0; s < world; ++s) total += n[s];
        std::vector<int64_t> cap(world);
        for (int r = 0; r < world; ++r)
            cap[r] = (next() % 8 == 0) ? (int64_t)(next() % (total + 1)) : total;  // sometimes tight
        std::vector<rsort_exchange_plan> xp(world);
        int verdict = -2;
        for (int me = 0; me < world; ++me) {
            const int st = rsort_multi_exchange_plan(world, me, buckets, counts.data(), &sp, cap.data(), &xp[me]);
            if (st != RSORT_OK && st != RSORT_ERR_CAPACITY) FAIL("status %d", st);
            if (verdict == -2) verdict = st;
            if (st != verdict) FAIL("ranks disagree on the verdict");
            if ((st == RSORT_ERR_CAPACITY) != (xp[me].over_capacity >= 0)) FAIL("over_capacity inconsistent");
            if (xp[me].total != total) FAIL("total");
        }
        for (int me = 0; me < world; ++me) {
            const rsort_exchange_plan &p = xp[me];
            int64_t off = 0;
            for (int r = 0; r < world; ++r) {
                if (p.send_off[r] != off || p.send_cnt[r] < 0) FAIL("sends of %d not contiguous", me);
                off += p.send_cnt[r];
                if (p.send_cnt[r] != xp[r].recv_cnt[me]) FAIL("%d->%d: send %lld, recv %lld", me, r,
                                                              (long long)p.send_cnt[r], (long long)xp[r].recv_cnt[me]);
            }
            if (off != n[me]) FAIL("sends of %d cover %lld of %lld", me, (long long)off, (long long)n[me]);
            int64_t ro = 0;
            for (int s = 0; s < world; ++s) {
                if (p.recv_off[s] != ro) FAIL("receives of %d not in source order", me);
                ro += p.recv_cnt[s];
            }
            if (ro != p.n_recv) FAIL("n_recv");
        }
        int64_t acc = 0, biggest = 0;
        for (int r = 0; r < world; ++r) {
            if (xp[r].offset != acc) FAIL("offset of %d", r);
            acc += xp[r].n_recv;
            for (int s = 0; s < world; ++s)
                if (s != r) biggest = std::max(biggest, xp[r].recv_cnt[s]);
            const bool over = xp[r].n_recv > cap[r];
            if (over && verdict != RSORT_ERR_CAPACITY) FAIL("rank %d over capacity not reported", r);
        }
        if (acc != total) FAIL("outputs sum to %lld of %lld", (long long)acc, (long long)total);
        if (xp[0].max_message != biggest) FAIL("max_message");
        // balanced cuts: boundary r inside its equal-keys bucket at clamp(r * total / world)
        for (int r = 1; r < world; ++r) {
            if (!sp.cut_inside[r]) continue;
            const int b = sp.cut_bucket[r];
            int64_t gb = 0, ge = 0;
            for (int bb = 0; bb <= b; ++bb)
                for (int s = 0; s < world; ++s) (bb < b ? gb : ge) += counts[(size_t)s * buckets + bb];
            ge += gb;
            const int64_t target = (int64_t)(((__int128)r * total) / world);
            const int64_t want = std::min(std::max(target, gb), ge);
            if (xp[r].offset != std::max(want, xp[r - 1].offset))
                FAIL("boundary %d at %lld, want %lld", r, (long long)xp[r].offset, (long long)want);
        }
        // the sampling plan
        std::vector<int64_t> nr(world);
        for (auto &x : nr) x = (next() % 5 == 0) ? 0 : (int64_t)(next() % 100000);
        rsort_sample_plan smp;
        const int64_t per = 1 + (int64_t)(next() % 5000);
        if (rsort_multi_sample_plan(world, nr.data(), per, &smp) != RSORT_OK) FAIL("sample plan");
        int64_t tot = 0, row = 1;
        for (int r = 0; r < world; ++r) {
            if (smp.count[r] * smp.stride < nr[r] || (smp.count[r] > 0 && (smp.count[r] - 1) * smp.stride >= nr[r]))
                FAIL("sample count of rank %d", r);
            tot += smp.count[r];
            row = std::max(row, smp.count[r]);
        }
        if (tot != smp.total || row != smp.row_len || smp.total > per * world + world) FAIL("sample totals");
        for (int i = 1; i < world; ++i) {
            const int64_t qi = rsort_multi_quantile_index(&smp, i);
            if (smp.total > 0 && (qi < 0 || qi >= smp.total)) FAIL("quantile index");
        }
    }
    printf("ok %d\n", cases);
    return 0;
}
