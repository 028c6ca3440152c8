// Backs DESIGN §3 "Pairs": one k = 8 pairs pass, 64-B-line rs_scatter_lines vs 128-B-line rs_scatter_pairs, with per-phase cycles.
// pairs_lab.hip -- development harness (not part of the library), backing DESIGN §3 "Pairs": one
// k = 8 pairs pass (2^lg pairs, 8192-pair tiles, 256 fixed chunks) through the 64-B-line pairs kernel
// (rs_scatter_lines<8, 512, 16, 16, true, ...>) and the 128-B-line one (rs_scatter_pairs), plain and
// clustered-input (CL) ranking, timed with HIP events and checked equal; per-phase s_memtime cycles
// per tile of rs_scatter_pairs (RS_STAMP, thread 0 of each workgroup).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cuda.radixsort_amd/csrc \
//         dev/pairs_lab.hip -o dev/pairs_lab && dev/pairs_lab [lg=30]
//   PL_ZIPF=1: Zipf(s=1) keys over 2^20 ranks (the C4 workload); PL_PASS=1: time pass 1 (digit 1) on
//   pass 0's output (clustered for Zipf keys); PL_REPS=n.
#define RSORT_STAMPS
#define RSORT_LAB_HOOKS "../../dev/lab_hooks.hpp"
#include "../cuda.radixsort_amd/csrc/rsort_kernels.hip"
#include "pairs_variants.hpp"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

using namespace rsort;

// the sequential-staging variant's own plan: 4096-pair tiles, 512 fixed chunks (two workgroups per CU)
static ScatterArgs g_sb2;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

static int env_int(const char *n, int d) {
    const char *e = getenv(n);
    return e ? atoi(e) : d;
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = 1ull << lg;
    const int zipf = env_int("PL_ZIPF", 0), pass = env_int("PL_PASS", 0), reps = env_int("PL_REPS", 5);
    constexpr uint32_t R = 256, TILE = 8192, CH = 256;
    const uint64_t tiles = (n + TILE - 1) / TILE, tpc = (tiles + CH - 1) / CH;
    const uint64_t chunk_keys = tpc * TILE;
    const uint32_t chunks = (uint32_t)((tiles + tpc - 1) / tpc);
    uint32_t *k0, *v0, *ka, *va, *kb, *vb, *table, *bsums, *cdf;
    unsigned long long *stamps;
    CK(hipMalloc(&k0, n * 4));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&ka, n * 4));
    CK(hipMalloc(&va, n * 4));
    CK(hipMalloc(&kb, n * 4));
    CK(hipMalloc(&vb, n * 4));
    CK(hipMalloc(&table, R * chunks * 4));
    constexpr uint32_t TILE2 = 4096, CH2 = 512;
    const uint64_t tiles2 = (n + TILE2 - 1) / TILE2, tpc2 = (tiles2 + CH2 - 1) / CH2;
    const uint64_t chunk_keys2 = tpc2 * TILE2;
    const uint32_t chunks2 = (uint32_t)((tiles2 + tpc2 - 1) / tpc2);
    uint32_t *table2;
    CK(hipMalloc(&table2, R * chunks2 * 4));
    CK(hipMalloc(&bsums, 4096));
    CK(hipMalloc(&stamps, chunks * 8 * 8));
    CK(hipMalloc(&cdf, (1u << 20) * 4));
    if (zipf) {  // the workload of tests/_util.py zipf_cdf_u32
        std::vector<double> c(1u << 20);
        double acc = 0;
        for (uint32_t r = 0; r < (1u << 20); ++r) c[r] = (acc += 1.0 / (r + 1.0));
        std::vector<uint32_t> t(1u << 20);
        for (uint32_t r = 0; r < (1u << 20); ++r) t[r] = (uint32_t)fmin(floor(c[r] / acc * 4294967296.0), 4294967295.0);
        t.back() = 0xFFFFFFFFu;
        CK(hipMemcpy(cdf, t.data(), t.size() * 4, hipMemcpyHostToDevice));
        rs_gen_zipf<<<65536, 256>>>(k0, n, 0x5EED, cdf, 1u << 20);
    } else {
        rs_gen_uniform<<<65536, 256>>>(k0, n, 0x5EED);
    }
    rs_gen_iota<<<65536, 256>>>(v0, n, 0);
    CK(hipDeviceSynchronize());

    auto table_for = [&](const uint32_t *keys, uint32_t shift, uint32_t *table, uint64_t chunk_keys, uint32_t chunks) {
        HistArgs h{};
        h.keys = keys;
        h.table = table;
        h.n = n;
        h.chunk_keys = chunk_keys;
        h.num_chunks = chunks;
        h.shift = shift;
        h.vec = 1;
        h.split = 1;
        rs_histogram<8, 1024, kDigitShift, 1, 8><<<chunks, 1024>>>(h);
        ScanArgs sa{};
        sa.table = table;
        sa.block_sums = bsums;
        sa.m = (uint64_t)R * chunks;
        sa.nblocks = (uint32_t)((sa.m + kScanSegment - 1) / kScanSegment);
        rs_scan_reduce<<<sa.nblocks, kScanThreads>>>(sa);
        rs_scan_down<<<sa.nblocks, kScanThreads>>>(sa);
        CK(hipGetLastError());
    };
    auto args = [&](const uint32_t *ki, const uint32_t *vi, uint32_t *ko, uint32_t *vo, uint32_t shift) {
        ScatterArgs a{};
        a.kin = ki;
        a.vin = vi;
        a.kout = ko;
        a.vout = vo;
        a.table = table;
        a.n = n;
        a.chunk_keys = chunk_keys;
        a.num_chunks = chunks;
        a.shift = shift;
        return a;
    };
    const uint32_t *in_k = k0, *in_v = v0;
    uint32_t shift = 0;
    if (pass == 1) {  // pass 0 first (64-B kernel), into ka/va; time pass 1 on it
        table_for(k0, 0, table, chunk_keys, chunks);
        rs_scatter_lines<8, 512, 16, kLineKeysPairs, true, kDigitShift, 2><<<chunks, 512>>>(args(k0, v0, ka, va, 0));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(k0, ka, n * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(v0, va, n * 4, hipMemcpyDeviceToDevice));
        shift = 8;
    }
    table_for(in_k, shift, table, chunk_keys, chunks);
    table_for(in_k, shift, table2, chunk_keys2, chunks2);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.3f ms/pass  %6.1f GB/s (%.3f of 8 TB/s)\n", name, ms / reps, 16.0 * n / (ms / reps) / 1e6,
               16.0 * n / (ms / reps) / 1e6 / 8000.0);
        fflush(stdout);
    };
    printf("2^%d pairs, %s keys, pass %d, %u chunks x %llu tiles\n", lg, zipf ? "Zipf" : "uniform", pass, chunks,
           (unsigned long long)tpc);
    // every variant writes kb/vb; timed round-robin (PL_ROUNDS rounds of `reps` passes each, the
    // best round reported: clocks and thermals drift over a run) and checked against the first
    ScatterArgs sb = args(in_k, in_v, kb, vb, shift);
    sb.stamps = stamps;
    g_sb2 = sb;
    g_sb2.table = table2;
    g_sb2.chunk_keys = chunk_keys2;
    g_sb2.num_chunks = chunks2;
    g_sb2.stamps = nullptr;
    struct Var {
        const char *name;
        void (*launch)(const ScatterArgs &, uint32_t);
        float best;
        std::vector<unsigned long long> st;
    };
    std::vector<Var> vars = {
        {"rs_scatter_lines 64-B 512 x 16", [](const ScatterArgs &x, uint32_t g) {
             rs_scatter_lines<8, 512, 16, kLineKeysPairs, true, kDigitShift, 2><<<g, 512>>>(x); }, 1e9f, {}},
        {"rs_scatter_pairs 128-B 1024 x 8", [](const ScatterArgs &x, uint32_t g) {
             rs_scatter_pairs<8, 1024, 8><<<g, 1024>>>(x); }, 1e9f, {}},
        {"rs_scatter_pairs 128-B 1024 x 8, CL", [](const ScatterArgs &x, uint32_t g) {
             rs_scatter_pairs<8, 1024, 8, 1><<<g, 1024>>>(x); }, 1e9f, {}},
        {"rs_scatter_pairs 512 x 8 seq. staging, 512 ch", [](const ScatterArgs &x, uint32_t g) {
             (void)x; (void)g;
             rs_scatter_pairs_lab<8, 512, 8, 0, 1, 64><<<g_sb2.num_chunks, 512>>>(g_sb2); }, 1e9f, {}},
        {"rs_scatter_pairs 512 x 8 seq. staging CL", [](const ScatterArgs &x, uint32_t g) {
             (void)x; (void)g;
             rs_scatter_pairs_lab<8, 512, 8, 1, 1, 64><<<g_sb2.num_chunks, 512>>>(g_sb2); }, 1e9f, {}},
        {"rs_scatter_pairs 1024 x 8 seq. staging, 256 ch", [](const ScatterArgs &x, uint32_t g) {
             rs_scatter_pairs_lab<8, 1024, 8, 1, 1, 64><<<g, 1024>>>(x); }, 1e9f, {}},
    };
    const int rounds = env_int("PL_ROUNDS", 3);
    std::vector<uint32_t> refk(n), refv(n), gk(n), gv(n);
    bool all_eq = true;
    for (size_t i = 0; i < vars.size(); ++i) {  // correctness first (and warm-up)
        vars[i].launch(sb, chunks);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(i == 0 ? refk.data() : gk.data(), kb, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(i == 0 ? refv.data() : gv.data(), vb, n * 4, hipMemcpyDeviceToHost));
        if (i > 0 && (memcmp(refk.data(), gk.data(), n * 4) || memcmp(refv.data(), gv.data(), n * 4))) {
            printf("  %s: OUTPUT DIFFERS\n", vars[i].name);
            all_eq = false;
        }
    }
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vars) {
            CK(hipMemset(stamps, 0, chunks * 8 * 8));
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) v.launch(sb, chunks);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            if (ms < v.best) {
                v.best = ms;
                v.st.resize(chunks * 8);
                CK(hipMemcpy(v.st.data(), stamps, chunks * 8 * 8, hipMemcpyDeviceToHost));
            }
        }
    for (auto &v : vars) {
        printf("%-46s %8.3f ms/pass  %6.1f GB/s (%.3f of 8 TB/s)", v.name, v.best, 16.0 * n / v.best / 1e6,
               16.0 * n / v.best / 1e6 / 8000.0);
        double tot = 0;
        for (uint32_t c = 0; c < chunks; ++c) tot += (double)v.st[c * 8];
        if (tot > 0) {  // rs_scatter_pairs: per-phase cycles per tile (thread 0, mean over chunks)
            printf("  cycles/tile (sync, seg-barrier, rec, stage, out, rank, seg-after-scan, seg-to-scan):");
            for (int i = 0; i < 8; ++i) {
                double s2 = 0;
                for (uint32_t c = 0; c < chunks; ++c) s2 += (double)v.st[c * 8 + i];
                printf(" %.0f", s2 / chunks / tpc);
            }
        }
        printf("\n");
    }
    printf("  outputs equal: %s\n", all_eq ? "yes" : "NO");
    const bool eq_k = all_eq;
    return eq_k ? 0 : 3;
}
