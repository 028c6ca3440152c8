// rsort_multi.cpp -- the multi-GPU sort (C ABI): rsort_u32_multi over an RCCL communicator and
// rsort_u32_multi_transport over any rsort_transport (the in-process loopback below is one).
//
// No reference counterpart (the reference sorts on one GPU, Parallel7.cu:10/:697); this is
// SURVEY.md §8e / BASELINE config 5, the same protocol as cuda.radixsort_amd/multi.py (which
// drives the same pure planning functions through torch.distributed):
//   1. all-gather every rank's key count; the sampling plan (rsort_multi_sample_plan)
//   2. a regular sample of the local keys, all-gathered, sorted on the device: the world - 1
//      global quantile keys (exact key values, not bin edges)
//   3. splitters with an equal-keys bucket per hot quantile key (rsort_multi_splitters_make_hot), a
//      stable partition of the local keys into those buckets
//   4. all-gather of the bucket counts and capacities; the exchange plan (rsort_multi_exchange_plan)
//      -- identical on every rank, so a capacity error is returned by all ranks together before
//      any key moves
//   5. ONE exchange: the rank's own range by a device copy, every other message point to point
//      (each pair of GPUs on its own xGMI link), cut into equal rounds of <= 2^28 keys
//   6. local LSD sort of what arrived, in place.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "rsort.h"
#include "rsort_internal.hpp"

using namespace rsort;

namespace {

constexpr int kMaxRanks = RSORT_MAX_RANKS;
constexpr int kMaxBuckets = 2 * kMaxRanks;
// total sample budget over all ranks: quantile error ~ sqrt(1/4/2^20) of the keys (0.05 %)
constexpr int64_t kSampleBudget = (int64_t)1 << 20;
// keys per message of one exchange round (1 GiB): this RCCL (2.26, ROCm 7) leaves the second half
// of an all_to_all / send message of >= 2 GiB unwritten without an error (dev/a2a_lab.py); 1 GiB
// messages arrive whole
constexpr int64_t kMaxPiece = (int64_t)1 << 28;
std::atomic<int64_t> g_piece{kMaxPiece};  // rsort_set_exchange_piece (tests force several rounds)
std::atomic<int> g_multi_opts{0};         // rsort_set_multi_options
std::atomic<int> g_multi_prof{0};         // rsort_multi_set_profiling
std::atomic<int> g_fail_rank{-1}, g_fail_stage{0}, g_fail_status{0};  // rsort_multi_inject_failure (tests)
int injected(int rank, int stage) {
    return (g_fail_rank.load() == rank && g_fail_stage.load() == stage) ? g_fail_status.load() : RSORT_OK;
}
// the calling thread's last profiled multi-GPU sort (the loopback tests run one rank per thread)
thread_local rsort_multi_stats t_stats;
thread_local bool t_stats_valid = false;

// hipEvents at the phase boundaries of one multi-GPU sort, on the caller's stream (profiling only)
struct MultiTimer {
    enum { kStart, kPlan, kPartition, kExchange, kEnd, kMarks };
    bool on = false;
    hipStream_t s;
    hipEvent_t ev[kMarks] = {};
    bool marked[kMarks] = {};
    MultiTimer(bool enable, hipStream_t stream) : s(stream) {
        if (!enable) return;
        on = true;
        for (auto &e : ev)
            if (hipEventCreate(&e) != hipSuccess) {
                e = nullptr;
                on = false;
            }
    }
    ~MultiTimer() {
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    void mark(int i) {
        if (on && hipEventRecord(ev[i], s) == hipSuccess) marked[i] = true;
    }
    double ms(int a, int b) const {
        float t = 0.f;
        if (!marked[a] || !marked[b] || hipEventElapsedTime(&t, ev[a], ev[b]) != hipSuccess) return 0.0;
        return t;
    }
    // waits for the sort to finish (profiling makes the call synchronous) and keeps the record
    int finish(rsort_multi_stats &st) {
        if (!on) return RSORT_OK;
        mark(kEnd);
        if (hipEventSynchronize(ev[kEnd]) != hipSuccess) return RSORT_ERR_HIP;
        // phases without a mark of their own (the direct world-1 sort) take the time up to the next
        int prev = kStart;
        double *out[kMarks] = {nullptr, &st.ms_plan, &st.ms_partition, &st.ms_exchange, &st.ms_local_sort};
        for (int i = kPlan; i < kMarks; ++i) {
            if (!marked[i]) continue;
            *out[i] = ms(prev, i);
            prev = i;
        }
        st.ms_total = ms(kStart, kEnd);
        t_stats = st;
        t_stats_valid = true;
        return RSORT_OK;
    }
};

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// step 1's all-gathered words per rank: key count, values flags, local status
constexpr size_t kNWords = 3;

struct MultiCarve {
    uint32_t *part_k, *part_v;
    uint64_t *n_send, *n_all;      // [kNWords], [world][kNWords]
    uint64_t *c_send, *c_all;      // [kMaxBuckets + 2], [world][kMaxBuckets + 2]: counts, capacity, status
    uint32_t *starts;              // [kMaxBuckets + 1]
    uint32_t *samp_send, *samp_all;  // [kSampleBudget + 1], [world][...]: the sample row + the status
    size_t control_bytes;          // the buffers above part_k
    void *sub;                     // partition, sample sort and local sort, in turn
    size_t sub_bytes;
};

int64_t samples_per_rank(int world) { return std::max<int64_t>(1, kSampleBudget / world); }

size_t sub_bytes(int64_t n, int64_t cap, int k, int pairs, int world) {
    (void)world;
    size_t a = rsort_partition_workspace_size(n, kMaxSplitters + 1, pairs);  // (any bucket count: overlap mode)
    // the gathered sample: world rows of at most kSampleBudget samples
    size_t b = rsort_workspace_size(world * kSampleBudget, 8, 0) + ((size_t)4 << 8 << 12);
    // the received count is only known later; a smaller n can pick a geometry with a larger
    // chunk table (<= 2^k x 4096 entries), or a digit-group plan where cap's is not, so leave room
    // for both
    size_t c = rsort_workspace_size(std::max<int64_t>(cap, 1), k, pairs) + ((size_t)4 << k << 12) +
               (k == kJointBits ? kJointExtraBytes : 0);
    return std::max(a, std::max(b, c));
}

size_t multi_bytes(int64_t n, int64_t cap, int k, int pairs, int world, MultiCarve *mc, void *base) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al256(bytes);
        return (char *)base + o;
    };
    MultiCarve m{};
    // the collectives' small buffers first: a rank whose workspace is too small for the rest still
    // takes part in them (with its error status, so every rank returns it together)
    m.n_send = (uint64_t *)take(kNWords * 8);
    m.n_all = (uint64_t *)take((size_t)kMaxRanks * kNWords * 8);
    m.c_send = (uint64_t *)take((size_t)(kMaxBuckets + 2) * 8);
    m.c_all = (uint64_t *)take((size_t)kMaxRanks * (kMaxBuckets + 2) * 8);
    m.starts = (uint32_t *)take((size_t)(kMaxBuckets + 1) * 4);
    m.samp_send = (uint32_t *)take((size_t)(kSampleBudget + 1) * 4);
    m.samp_all = (uint32_t *)take((size_t)world * (kSampleBudget + 1) * 4);
    m.control_bytes = off;
    m.part_k = (uint32_t *)take((size_t)n * 4);
    m.part_v = pairs ? (uint32_t *)take((size_t)n * 4) : nullptr;
    m.sub_bytes = sub_bytes(n, cap, k, pairs, world);
    m.sub = take(m.sub_bytes);
    if (mc) *mc = m;
    return off;
}

int hip_st(hipError_t e) { return e == hipSuccess ? RSORT_OK : RSORT_ERR_HIP; }

// A second stream per device (with its two events) for work that overlaps the exchange: created on
// first use, kept for the process. Concurrent multi-GPU sorts on one device (the loopback tests'
// ranks) each take their own from a small pool.
struct SideStream {
    int device;
    bool busy;
    hipStream_t s;
    hipEvent_t ready, done;
};
std::mutex g_side_mu;
std::vector<SideStream *> g_side;

SideStream *side_stream() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_side_mu);
    for (SideStream *x : g_side)
        if (x->device == dev && !x->busy) {
            x->busy = true;
            return x;
        }
    SideStream *x = new (std::nothrow) SideStream{dev, true, nullptr, nullptr, nullptr};
    if (!x) return nullptr;
    if (hipStreamCreateWithFlags(&x->s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&x->ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->done, hipEventDisableTiming) != hipSuccess) {
        delete x;  // (a partly created stream/event leaks: a HIP failure this early is terminal anyway)
        return nullptr;
    }
    g_side.push_back(x);
    return x;
}

void side_release(SideStream *x) {
    if (!x) return;
    std::lock_guard<std::mutex> g(g_side_mu);
    x->busy = false;
}

// ------------------------------------------------------------------------------ RCCL transport
// Every RCCL step is bounded: RCCL itself never times out, so a peer that died or
// never joined would leave this rank's kernels spinning and its host waiting forever. Each step's
// calls are completed (a non-blocking communicator returns ncclInProgress until they are), then the
// step's stream work is polled to completion; past the deadline, or on an asynchronous RCCL error,
// the communicator is aborted (ncclCommAbort also stops its kernels) and RSORT_ERR_COMM returned.
std::atomic<int> g_comm_timeout_ms{300000};  // rsort_set_comm_timeout
std::mutex g_aborted_mu;
// communicators a timeout aborted and nobody has released yet: rsort_u32_multi refuses them and
// rsort_rccl_comm_destroy only forgets them (ncclCommAbort freed them). An address leaves the list when
// destroy is called for it and when rsort_rccl_comm_init hands it out again for a new, live communicator
// (freed communicators' addresses are reused, so a stale entry would refuse a live one)
std::vector<void *> g_aborted;

void comm_forget(ncclComm_t c) {
    std::lock_guard<std::mutex> g(g_aborted_mu);
    g_aborted.erase(std::remove(g_aborted.begin(), g_aborted.end(), (void *)c), g_aborted.end());
}

bool comm_aborted(ncclComm_t c) {
    std::lock_guard<std::mutex> g(g_aborted_mu);
    return std::find(g_aborted.begin(), g_aborted.end(), (void *)c) != g_aborted.end();
}

int comm_abort(ncclComm_t c) {
    {
        std::lock_guard<std::mutex> g(g_aborted_mu);
        if (std::find(g_aborted.begin(), g_aborted.end(), (void *)c) != g_aborted.end()) return RSORT_ERR_COMM;
        g_aborted.push_back((void *)c);
    }
    (void)ncclCommAbort(c);
    return RSORT_ERR_COMM;
}

using Clock = std::chrono::steady_clock;

// r == ncclInProgress (a non-blocking communicator): poll until the call has completed
ncclResult_t nb_complete(ncclComm_t c, ncclResult_t r, Clock::time_point deadline) {
    while (r == ncclInProgress) {
        if (Clock::now() > deadline) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return ncclInternalError;
    }
    return r;
}

// the step's calls returned `r`; now wait (bounded) for its work on `s`
int rccl_finish(ncclComm_t c, ncclResult_t r, hipStream_t s, Clock::time_point deadline) {
    r = nb_complete(c, r, deadline);
    if (r != ncclSuccess) return comm_abort(c);
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return RSORT_ERR_HIP;
    int st = hipEventRecord(ev, s) == hipSuccess ? RSORT_OK : RSORT_ERR_HIP;
    for (int spin = 0; st == RSORT_OK; ++spin) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) {
            st = RSORT_ERR_HIP;
            break;
        }
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(c, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress) ||
            Clock::now() > deadline) {
            st = comm_abort(c);
            break;
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    (void)hipEventDestroy(ev);
    return st;
}

Clock::time_point comm_deadline() { return Clock::now() + std::chrono::milliseconds(g_comm_timeout_ms.load()); }

struct RcclCtx {
    ncclComm_t comm;
};

int rccl_allgather(void *ctx, const void *d_send, void *d_recv, size_t bytes, void *stream) {
    ncclComm_t comm = static_cast<RcclCtx *>(ctx)->comm;
    const Clock::time_point dl = comm_deadline();
    return rccl_finish(comm, ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, (hipStream_t)stream),
                       (hipStream_t)stream, dl);
}

int rccl_exchange(void *ctx, void *const *d_send, const size_t *send_bytes, void *const *d_recv,
                  const size_t *recv_bytes, void *stream) {
    ncclComm_t comm = static_cast<RcclCtx *>(ctx)->comm;
    int world = 0, me = 0;
    if (ncclCommCount(comm, &world) != ncclSuccess || ncclCommUserRank(comm, &me) != ncclSuccess) return RSORT_ERR_COMM;
    hipStream_t s = (hipStream_t)stream;
    const Clock::time_point dl = comm_deadline();
    // every call inside the group is checked; the group is always closed (an open group would
    // leave the communicator unusable), and the first failure is returned
    ncclResult_t first = ncclGroupStart();
    if (first != ncclSuccess) return comm_abort(comm);
    for (int p = 0; p < world; ++p) {
        if (p == me) continue;
        if (send_bytes[p]) {
            const ncclResult_t r = ncclSend(d_send[p], send_bytes[p], ncclUint8, p, comm, s);
            if (first == ncclSuccess) first = r;
        }
        if (recv_bytes[p]) {
            const ncclResult_t r = ncclRecv(d_recv[p], recv_bytes[p], ncclUint8, p, comm, s);
            if (first == ncclSuccess) first = r;
        }
    }
    const ncclResult_t e = ncclGroupEnd();
    if (first == ncclSuccess || first == ncclInProgress) first = e;
    return rccl_finish(comm, first, s, dl);
}

// ------------------------------------------------------------------------------ loopback transport
// World of `world` ranks in one process (one thread per rank, any devices with peer access, or one
// device): collectives through a host rendezvous and device-to-device copies. Test transport for
// the multi-GPU path on a one-GPU box (RCCL refuses two ranks on one device: "Duplicate GPU
// detected"); every wait is bounded so a protocol bug ends in RSORT_ERR_COMM, not a hang.
struct LoopbackGroup;
struct LoopbackCtx {
    LoopbackGroup *g;
    int rank;
};

struct LoopbackGroup {
    int world;
    LoopbackCtx ctx[kMaxRanks];
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    bool broken = false;
    // posted by each rank between two barriers
    const void *ag_src[kMaxRanks];
    size_t ag_bytes[kMaxRanks];
    void *const *ex_send[kMaxRanks];
    const size_t *ex_send_bytes[kMaxRanks];

    // returns false on timeout (and marks the group broken so every rank fails fast)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen || broken; });
        if (!ok || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

int lb_allgather(void *ctx, const void *d_send, void *d_recv, size_t bytes, void *stream) {
    LoopbackCtx *c = static_cast<LoopbackCtx *>(ctx);
    LoopbackGroup *g = c->g;
    hipStream_t s = (hipStream_t)stream;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;  // d_send is ready
    g->ag_src[c->rank] = d_send;
    g->ag_bytes[c->rank] = bytes;
    if (!g->barrier()) return RSORT_ERR_COMM;
    int st = RSORT_OK;
    for (int r = 0; r < g->world && !st; ++r) {
        if (g->ag_bytes[r] != bytes) st = RSORT_ERR_COMM;
        else if (bytes && hipMemcpyAsync((char *)d_recv + (size_t)r * bytes, g->ag_src[r], bytes,
                                         hipMemcpyDeviceToDevice, s) != hipSuccess)
            st = RSORT_ERR_HIP;
    }
    if (!st && hipStreamSynchronize(s) != hipSuccess) st = RSORT_ERR_HIP;
    if (!g->barrier()) return RSORT_ERR_COMM;  // nobody reuses its send buffer before all have copied
    return st;
}

int lb_exchange(void *ctx, void *const *d_send, const size_t *send_bytes, void *const *d_recv,
                const size_t *recv_bytes, void *stream) {
    LoopbackCtx *c = static_cast<LoopbackCtx *>(ctx);
    LoopbackGroup *g = c->g;
    hipStream_t s = (hipStream_t)stream;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    g->ex_send[c->rank] = d_send;
    g->ex_send_bytes[c->rank] = send_bytes;
    if (!g->barrier()) return RSORT_ERR_COMM;
    int st = RSORT_OK;
    for (int p = 0; p < g->world && !st; ++p) {
        if (p == c->rank) continue;
        // what p sends to me must be what I expect to receive from p
        if (g->ex_send_bytes[p][c->rank] != recv_bytes[p]) st = RSORT_ERR_COMM;
        else if (recv_bytes[p] && hipMemcpyAsync(d_recv[p], g->ex_send[p][c->rank], recv_bytes[p],
                                                 hipMemcpyDeviceToDevice, s) != hipSuccess)
            st = RSORT_ERR_HIP;
    }
    if (!st && hipStreamSynchronize(s) != hipSuccess) st = RSORT_ERR_HIP;
    if (!g->barrier()) return RSORT_ERR_COMM;
    return st;
}

// ------------------------------------------------------------------------------ host transport
// rsort_host_transport_wrap: device bytes staged through host buffers for a host-memory transport
struct HostCtx {
    rsort_host_transport host;
    std::vector<char> send, recv;
};

int host_allgather(void *ctx, const void *d_send, void *d_recv, size_t bytes, void *stream) {
    HostCtx *c = static_cast<HostCtx *>(ctx);
    hipStream_t s = (hipStream_t)stream;
    const size_t world = (size_t)c->host.world;
    c->send.resize(std::max<size_t>(bytes, 1));
    c->recv.resize(std::max<size_t>(world * bytes, 1));
    if (bytes && hipMemcpyAsync(c->send.data(), d_send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        return RSORT_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    const int st = c->host.allgather(c->host.ctx, c->send.data(), c->recv.data(), bytes);
    if (st) return st;
    if (bytes && hipMemcpyAsync(d_recv, c->recv.data(), world * bytes, hipMemcpyHostToDevice, s) != hipSuccess)
        return RSORT_ERR_HIP;
    return hip_st(hipStreamSynchronize(s));
}

int host_exchange(void *ctx, void *const *d_send, const size_t *send_bytes, void *const *d_recv,
                  const size_t *recv_bytes, void *stream) {
    HostCtx *c = static_cast<HostCtx *>(ctx);
    hipStream_t s = (hipStream_t)stream;
    const int world = c->host.world;
    size_t so[kMaxRanks + 1] = {0}, ro[kMaxRanks + 1] = {0};
    for (int p = 0; p < world; ++p) {
        so[p + 1] = so[p] + send_bytes[p];
        ro[p + 1] = ro[p] + recv_bytes[p];
    }
    c->send.resize(std::max<size_t>(so[world], 1));
    c->recv.resize(std::max<size_t>(ro[world], 1));
    void *hs[kMaxRanks], *hr[kMaxRanks];
    for (int p = 0; p < world; ++p) {
        hs[p] = c->send.data() + so[p];
        hr[p] = c->recv.data() + ro[p];
        if (send_bytes[p] && hipMemcpyAsync(hs[p], d_send[p], send_bytes[p], hipMemcpyDeviceToHost, s) != hipSuccess)
            return RSORT_ERR_HIP;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
    const int st = c->host.exchange(c->host.ctx, hs, send_bytes, hr, recv_bytes);
    if (st) return st;
    for (int p = 0; p < world; ++p)
        if (recv_bytes[p] && hipMemcpyAsync(d_recv[p], hr[p], recv_bytes[p], hipMemcpyHostToDevice, s) != hipSuccess)
            return RSORT_ERR_HIP;
    return hip_st(hipStreamSynchronize(s));
}

// ------------------------------------------------------------------------------ the sort
int d2h(void *h, const void *d, size_t bytes, hipStream_t s) {
    if (hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return RSORT_ERR_HIP;
    return hip_st(hipStreamSynchronize(s));
}

int multi_sort(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n, uint32_t *d_keys_out, uint32_t *d_vals_out,
               int64_t capacity, int64_t *out_n, int64_t *out_offset, int k_bits, const rsort_transport *tr,
               void *d_workspace, size_t workspace_bytes, hipStream_t s) {
    // What every collective needs: a transport, this rank's place in it and the small control
    // buffers. Without them a rank cannot even tell its peers it failed (caller error).
    if (!tr || !tr->allgather || !tr->exchange || !d_workspace) return RSORT_ERR_ARG;
    const int world = tr->world, me = tr->rank;
    if (world < 1 || world > kMaxRanks || me < 0 || me >= world) return RSORT_ERR_ARG;
    const bool sizes_ok = n >= 0 && n < ((int64_t)1 << 32) && capacity >= 0 && capacity < ((int64_t)1 << 32);
    // a rank sorts pairs when it passes values or a values output (a rank with no keys may pass
    // an empty, NULL values input); the ranks agree on it in step 1
    const int pairs = (d_vals != nullptr || d_vals_out != nullptr) ? 1 : 0;
    MultiCarve m;
    const size_t need = multi_bytes(sizes_ok ? n : 0, sizes_ok ? capacity : 0, k_bits, pairs, world, &m, d_workspace);
    if (workspace_bytes < m.control_bytes) return RSORT_ERR_WORKSPACE;
    // Every other local failure is carried to the peers in the next all-gather (a status word per
    // rank) and returned by every rank together -- the lowest rank's status first -- instead of
    // leaving the peers waiting in a collective this rank never joins (a rank that dies instead is
    // caught by the RCCL transport's bounded waits: rccl_finish).
    int local = RSORT_OK;
    if (k_bits < kMinBits || k_bits > kMaxBits) local = RSORT_ERR_BITS;
    else if (!sizes_ok) local = RSORT_ERR_SIZE;
    else if (!out_n || !out_offset || (n > 0 && !d_keys) || (capacity > 0 && !d_keys_out)) local = RSORT_ERR_ARG;
    else if (workspace_bytes < need) local = RSORT_ERR_WORKSPACE;
    if (local != RSORT_OK) n = 0;  // (nothing below reads the keys of a failed rank)
    int st;
    const int opts = g_multi_opts.load();
    rsort_multi_stats stats;
    memset(&stats, 0, sizeof(stats));
    stats.world = world;
    stats.rank = me;
    stats.n_in = n;
    stats.bytes_per_key = pairs ? 8 : 4;
    MultiTimer timer(g_multi_prof.load() != 0, s);
    timer.mark(MultiTimer::kStart);
    if (world == 1 && !(opts & RSORT_MULTI_FULL)) {
        // one rank: the partition would be one bucket (a copy) and the exchange a self copy, so the
        // keys go straight through the local sort (same output, no peers to agree with)
        if (local != RSORT_OK) return local;
        if (n > capacity) return RSORT_ERR_CAPACITY;
        timer.mark(MultiTimer::kExchange);  // (nothing exchanged: the whole time is the local sort)
        if (n > 0) {
            rsort_plan p;
            if ((st = rsort_plan_make(n, k_bits, pairs, 0, &p))) return st;
            if ((st = rsort_sort_planned(&p, d_keys, d_vals, d_keys_out, d_vals_out, m.sub, m.sub_bytes, s))) return st;
        }
        *out_n = n;
        *out_offset = 0;
        stats.direct = 1;
        stats.halves = 1;
        stats.n_out = n;
        stats.send_keys[0] = stats.recv_keys[0] = n;
        return timer.finish(stats);
    }
    // RSORT_MULTI_OVERLAP: every rank's key range is cut in two (H = 2 virtual ranks per rank, the
    // planning functions run for world * H ranks); the lower half is exchanged first and sorted on a
    // side stream while the upper half is exchanged
    // (automatic: 2 <= world <= RSORT_MULTI_AUTO_OVERLAP_MAX_WORLD, rsort.h and DESIGN §5)
    const bool ov = (opts & RSORT_MULTI_OVERLAP) != 0 ||
                    (!(opts & RSORT_MULTI_NO_OVERLAP) && world <= RSORT_MULTI_AUTO_OVERLAP_MAX_WORLD);
    const int H = (ov && world >= 2 && 2 * world <= kMaxRanks) ? 2 : 1;
    const int V = world * H;
    auto first_status = [&](const uint64_t *words, size_t stride, size_t at) {
        for (int r = 0; r < world; ++r)
            if (words[(size_t)r * stride + at] != 0) return (int)words[(size_t)r * stride + at];
        return (int)RSORT_OK;
    };

    // 1. key counts, value flags and statuses -> sampling plan; a values mismatch between ranks is
    //    an argument error on every rank (all see the same flags)
    const uint64_t mine[kNWords] = {(uint64_t)n, (uint64_t)(pairs | (d_vals ? 2 : 0) | (d_vals_out ? 4 : 0)),
                                    (uint64_t)local};
    if (hipMemcpyAsync(m.n_send, mine, sizeof(mine), hipMemcpyHostToDevice, s) != hipSuccess) return RSORT_ERR_HIP;
    if ((st = tr->allgather(tr->ctx, m.n_send, m.n_all, sizeof(mine), s))) return st;
    uint64_t nf[kNWords * kMaxRanks];
    if ((st = d2h(nf, m.n_all, (size_t)world * sizeof(mine), s))) return st;
    if ((st = first_status(nf, kNWords, 2))) return st;
    int64_t n_all[kMaxRanks] = {0};  // per virtual rank: rank r's keys at r * H, none at the others
    bool any_pairs = false, bad = false;
    for (int r = 0; r < world; ++r) {
        n_all[r * H] = (int64_t)nf[kNWords * r];
        any_pairs |= (nf[kNWords * r + 1] & 1) != 0;
    }
    for (int r = 0; r < world && any_pairs; ++r)
        bad |= !(nf[kNWords * r + 1] & 4) || ((int64_t)nf[kNWords * r] > 0 && !(nf[kNWords * r + 1] & 2));
    if (bad) return RSORT_ERR_ARG;
    rsort_sample_plan sp;
    if ((st = rsort_multi_sample_plan(V, n_all, samples_per_rank(V), &sp))) return st;
    if (sp.row_len > kSampleBudget) return RSORT_ERR_ARG;  // cannot happen: budget / V per virtual rank

    // 2. sample (+ this rank's status in the row's last word), gather, sort on the device, read
    //    the quantile keys
    const size_t row = (size_t)sp.row_len + 1;
    if (launch_sample(d_keys, (uint64_t)n, (uint64_t)sp.stride, (uint64_t)sp.count[me * H], (uint64_t)sp.row_len,
                      m.samp_send, s) != hipSuccess)
        local = RSORT_ERR_HIP;
    const uint32_t lst = (uint32_t)local;
    if (hipMemcpyAsync(m.samp_send + sp.row_len, &lst, 4, hipMemcpyHostToDevice, s) != hipSuccess) return RSORT_ERR_HIP;
    if ((st = tr->allgather(tr->ctx, m.samp_send, m.samp_all, row * 4, s))) return st;
    {
        uint32_t sts[kMaxRanks];
        for (int r = 0; r < world; ++r)
            if (hipMemcpyAsync(&sts[r], m.samp_all + (size_t)r * row + sp.row_len, 4, hipMemcpyDeviceToHost, s) !=
                hipSuccess)
                return RSORT_ERR_HIP;
        if (hipStreamSynchronize(s) != hipSuccess) return RSORT_ERR_HIP;
        for (int r = 0; r < world; ++r)
            if (sts[r]) return (int)sts[r];
    }
    uint32_t q[kMaxRanks] = {0};
    int hot[kMaxRanks] = {0};
    if (V > 1 && sp.total > 0) {
        // the rows (each followed by its status word) sorted as one array: the status words are 0
        // and sort first, so the quantile positions move up by world (and the rows' padding, 0xFFFFFFFF,
        // sorts after the sp.total samples)
        const int64_t ns = (int64_t)world * (int64_t)row;
        profile_pause(1);  // (its passes are part of the plan phase, not the measured local sort)
        local = rsort_u32_device(m.samp_all, m.samp_all, ns, 8, m.sub, m.sub_bytes, s);
        profile_pause(-1);
        // each quantile key and the samples hot_reach away on both sides: the key is hot (its own
        // equal-keys bucket, rsort_multi_splitters_make_hot) when either is the same key
        const int64_t L = std::max<int64_t>(1, sp.total / ((int64_t)V * 128));
        uint32_t nb[kMaxRanks][2];
        for (int i = 1; i < V && !local; ++i) {
            const int64_t qi = rsort_multi_quantile_index(&sp, i);
            const int64_t at[3] = {qi, qi - L, qi + L};
            uint32_t *dst[3] = {&q[i - 1], &nb[i - 1][0], &nb[i - 1][1]};
            nb[i - 1][0] = nb[i - 1][1] = 0;
            for (int j = 0; j < 3 && !local; ++j) {
                if (at[j] < 0 || at[j] >= sp.total) continue;  // (a neighbour outside the samples: not hot there)
                if (hipMemcpyAsync(dst[j], m.samp_all + world + at[j], 4, hipMemcpyDeviceToHost, s) != hipSuccess)
                    local = RSORT_ERR_HIP;
            }
        }
        if (!local && hipStreamSynchronize(s) != hipSuccess) local = RSORT_ERR_HIP;
        for (int i = 1; i < V && !local; ++i) {
            const int64_t qi = rsort_multi_quantile_index(&sp, i);
            hot[i - 1] = (qi - L >= 0 && nb[i - 1][0] == q[i - 1]) || (qi + L < sp.total && nb[i - 1][1] == q[i - 1]);
        }
        if (!local) local = injected(me, 1);
        if (local) q[0] = 0xFFFFFFFFu;  // (a failed copy may leave partial quantiles: replaced below)
    }
    // From here a rank that failed since the last status exchange (the sample sort, a quantile copy)
    // still joins the next all-gather with a row of the same size as its peers' and its status in
    // it: it plans on placeholder quantiles (all 0, monotone) instead of its partial ones, and a
    // failure of the pure splitter planning is carried the same way instead of returned.
    if (local) {
        memset(q, 0, sizeof(q));
        memset(hot, 0, sizeof(hot));
    }
    rsort_multi_splitters spl;
    if ((st = rsort_multi_splitters_make_hot(V, q, hot, &spl))) {  // pure, identical on every healthy rank
        if (!local) local = st;
        memset(&spl, 0, sizeof(spl));
        spl.world = V;
    }
    timer.mark(MultiTimer::kPlan);

    // 3. stable partition into the splitters' buckets
    const int buckets = std::min(spl.nsplit + 1, kMaxSplitters + 1);
    if (spl.nsplit + 1 > kMaxSplitters + 1 && !local) local = RSORT_ERR_ARG;  // (pure: every rank alike)
    uint32_t starts[kMaxBuckets + 1] = {0};
    if (!local) local = injected(me, 2);
    if (!local)
        local = rsort_partition_device(d_keys, d_vals, m.part_k, m.part_v, n, spl.split, buckets, m.starts, m.sub,
                                       m.sub_bytes, s);
    if (!local) local = d2h(starts, m.starts, (size_t)(buckets + 1) * 4, s);
    if (!local) {  // the partition's self-check (its scatter's rank check): a failure stops every rank below
        int pf = 0;
        local = rsort_partition_check(n, buckets, d_vals != nullptr ? 1 : 0, m.sub, &pf, s);
        if (!local && pf) local = RSORT_ERR_CHECK;
    }

    // 4. count matrix + capacities + statuses -> the exchange plans (the same on every rank). The
    //    row has a fixed size whatever this rank's bucket count (a failed rank's may differ), so the
    //    all-gather always matches: counts in [0, buckets), capacity and status at fixed words.
    constexpr int kRow = kMaxBuckets + 2, kCapWord = kMaxBuckets, kStatusWord = kMaxBuckets + 1;
    uint64_t rowc[kRow] = {0};
    for (int b = 0; b < buckets && !local; ++b) rowc[b] = (uint64_t)(starts[b + 1] - starts[b]);
    rowc[kCapWord] = (uint64_t)capacity;
    rowc[kStatusWord] = (uint64_t)local;
    const size_t row_bytes = sizeof(rowc);
    if (hipMemcpyAsync(m.c_send, rowc, row_bytes, hipMemcpyHostToDevice, s) != hipSuccess) return RSORT_ERR_HIP;
    if ((st = tr->allgather(tr->ctx, m.c_send, m.c_all, row_bytes, s))) return st;
    uint64_t all[kMaxRanks * kRow];
    if ((st = d2h(all, m.c_all, (size_t)world * row_bytes, s))) return st;
    if ((st = first_status(all, (size_t)kRow, (size_t)kStatusWord))) return st;
    int64_t counts[kMaxRanks * kMaxBuckets] = {0}, caps[kMaxRanks], cap_of[kMaxRanks];
    for (int r = 0; r < world; ++r) {
        for (int b = 0; b < buckets; ++b) counts[r * H * buckets + b] = (int64_t)all[r * kRow + b];
        cap_of[r] = (int64_t)all[r * kRow + kCapWord];
        for (int h = 0; h < H; ++h) caps[r * H + h] = cap_of[r];  // (the halves' sum is checked below)
    }
    // every virtual rank's plan: this rank sends as virtual rank me * H and receives as me * H + h;
    // the capacity check is on each rank's total
    rsort_exchange_plan xv[kMaxRanks];
    for (int v = 0; v < V; ++v) {
        st = rsort_multi_exchange_plan(V, v, buckets, counts, &spl, caps, &xv[v]);
        if (st != RSORT_OK && st != RSORT_ERR_CAPACITY) return st;
    }
    for (int r = 0; r < world; ++r) {
        int64_t tot = 0;
        for (int h = 0; h < H; ++h) tot += xv[r * H + h].n_recv;
        if (tot > cap_of[r]) return RSORT_ERR_CAPACITY;
    }
    const rsort_exchange_plan &xs = xv[me * H];  // (all sends of this rank)

    // 5-6. per half: the exchange (the own range by a device copy on a side stream beside the
    //      messages, which the transport moves on `s`; the rest in equal rounds of <= the piece
    //      limit), then the local sort of what arrived, in place. With two halves the first half's
    //      sort runs on the side stream while the second half is exchanged.
    int64_t rounds = 0, piece = 0;
    if ((st = rsort_multi_exchange_rounds(xs.max_message, g_piece.load(), &rounds, &piece))) return st;
    timer.mark(MultiTimer::kPartition);
    stats.halves = H;
    stats.rounds = rounds;
    for (int p = 0; p < world; ++p)
        for (int h = 0; h < H; ++h) {
            stats.send_keys[p] += xs.send_cnt[p * H + h];
            stats.recv_keys[p] += xv[me * H + h].recv_cnt[p * H];
        }
    SideStream *side = side_stream();
    // On EVERY return while the side stream holds work (an own-range copy, the lower half's sort)
    // `s` first waits for it, so a caller that synchronises `s` after an error never frees buffers
    // a side-stream kernel still writes; only then does the stream go back to the pool (a later user
    // enqueues behind the work anyway, and the wait already captured the event's state).
    struct SideGuard {
        SideStream *x;
        hipStream_t s;
        bool pending = false;  // the side stream holds work `s` must wait for
        ~SideGuard() {
            if (x && pending) (void)hipStreamWaitEvent(s, x->done, 0);
            side_release(x);
        }
    } side_guard{side, s};
    bool &side_pending = side_guard.pending;
    int64_t base = 0;
    for (int h = 0; h < H; ++h) {
        const rsort_exchange_plan &xd = xv[me * H + h];
        const int own_dst = me * H + h, own_src = me * H;
        if (xs.send_cnt[own_dst] != xd.recv_cnt[own_src]) return RSORT_ERR_ARG;
        uint32_t *ok = d_keys_out + base, *ov = pairs ? d_vals_out + base : nullptr;
        const int64_t own = xs.send_cnt[own_dst];
        if (own > 0) {
            hipStream_t cs = s;
            if (side && !side_pending && hipEventRecord(side->ready, s) == hipSuccess &&
                hipStreamWaitEvent(side->s, side->ready, 0) == hipSuccess)
                cs = side->s;
            if (hipMemcpyAsync(ok + xd.recv_off[own_src], m.part_k + xs.send_off[own_dst], (size_t)own * 4,
                               hipMemcpyDeviceToDevice, cs) != hipSuccess)
                return RSORT_ERR_HIP;
            if (pairs && hipMemcpyAsync(ov + xd.recv_off[own_src], m.part_v + xs.send_off[own_dst], (size_t)own * 4,
                                        hipMemcpyDeviceToDevice, cs) != hipSuccess)
                return RSORT_ERR_HIP;
            if (cs != s) {
                if (hipEventRecord(side->done, side->s) != hipSuccess) return RSORT_ERR_HIP;
                side_pending = true;
            }
        }
        for (int64_t rd = 0; rd < rounds; ++rd) {
            for (int arr = 0; arr < (pairs ? 2 : 1); ++arr) {
                uint32_t *src = arr ? m.part_v : m.part_k;
                uint32_t *dst = arr ? ov : ok;
                void *sp_[kMaxRanks], *rp_[kMaxRanks];
                size_t sb[kMaxRanks], rb[kMaxRanks];
                for (int p = 0; p < world; ++p) {
                    const int dv = p * H + h, sv = p * H;  // virtual destination / source
                    const int64_t a0 = std::min(xs.send_cnt[dv], rd * piece), a1 = std::min(xs.send_cnt[dv], (rd + 1) * piece);
                    const int64_t b0 = std::min(xd.recv_cnt[sv], rd * piece), b1 = std::min(xd.recv_cnt[sv], (rd + 1) * piece);
                    sp_[p] = src + xs.send_off[dv] + a0;
                    rp_[p] = dst + xd.recv_off[sv] + b0;
                    sb[p] = p == me ? 0 : (size_t)(a1 - a0) * 4;
                    rb[p] = p == me ? 0 : (size_t)(b1 - b0) * 4;
                }
                if ((st = tr->exchange(tr->ctx, sp_, sb, rp_, rb, s))) return st;
            }
        }
        // this half has arrived (on `s`, and its own range on the side stream); under the overlap the
        // exchange phase ends with the last message, before waiting for the lower half's sort
        if (h + 1 == H && H > 1) timer.mark(MultiTimer::kExchange);
        if (side_pending) {
            if (hipStreamWaitEvent(s, side->done, 0) != hipSuccess) return RSORT_ERR_HIP;
            side_pending = false;
        }
        if (h + 1 == H && H == 1) timer.mark(MultiTimer::kExchange);
        if (xd.n_recv > 0) {
            rsort_plan p;
            if ((st = rsort_plan_make(xd.n_recv, k_bits, pairs, 0, &p))) return st;
            hipStream_t ss = s;
            if (h + 1 < H && side && hipEventRecord(side->ready, s) == hipSuccess &&
                hipStreamWaitEvent(side->s, side->ready, 0) == hipSuccess)
                ss = side->s;  // sorted while the next half is exchanged on `s`
            if ((st = rsort_sort_planned(&p, ok, ov, ok, ov, m.sub, m.sub_bytes, ss))) return st;
            if (ss != s) {
                if (hipEventRecord(side->done, side->s) != hipSuccess) return RSORT_ERR_HIP;
                side_pending = true;  // (the next half's own copy then stays on `s`)
            }
        }
        base += xd.n_recv;
    }
    if (side_pending) {
        if (hipStreamWaitEvent(s, side->done, 0) != hipSuccess) return RSORT_ERR_HIP;
        side_pending = false;
    }
    *out_n = base;
    *out_offset = xv[me * H].offset;
    stats.n_out = base;
    return timer.finish(stats);
}

}  // namespace

extern "C" {

size_t rsort_multi_workspace_size(int64_t n, int64_t capacity, int k_bits, int pairs, int world) {
    if (n < 0 || capacity < 0 || world < 1 || world > kMaxRanks) return 0;
    return multi_bytes(n, capacity, k_bits, pairs ? 1 : 0, world, nullptr, nullptr);
}

int rsort_u32_multi_transport(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n, uint32_t *d_keys_out,
                              uint32_t *d_vals_out, int64_t capacity, int64_t *out_n, int64_t *out_offset, int k_bits,
                              const rsort_transport *transport, void *d_workspace, size_t workspace_bytes,
                              void *stream) {
    return multi_sort(d_keys, d_vals, n, d_keys_out, d_vals_out, capacity, out_n, out_offset, k_bits, transport,
                      d_workspace, workspace_bytes, (hipStream_t)stream);
}

int rsort_u32_multi(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n, uint32_t *d_keys_out,
                    uint32_t *d_vals_out, int64_t capacity, int64_t *out_n, int64_t *out_offset, int k_bits,
                    void *nccl_comm, void *d_workspace, size_t workspace_bytes, void *stream) {
    if (!nccl_comm) return RSORT_ERR_ARG;
    if (comm_aborted((ncclComm_t)nccl_comm)) return RSORT_ERR_COMM;  // (a timeout aborted it earlier)
    RcclCtx ctx{(ncclComm_t)nccl_comm};
    int world = 0, me = 0;
    if (ncclCommCount(ctx.comm, &world) != ncclSuccess || ncclCommUserRank(ctx.comm, &me) != ncclSuccess)
        return RSORT_ERR_COMM;
    rsort_transport tr{&ctx, world, me, rccl_allgather, rccl_exchange};
    return multi_sort(d_keys, d_vals, n, d_keys_out, d_vals_out, capacity, out_n, out_offset, k_bits, &tr,
                      d_workspace, workspace_bytes, (hipStream_t)stream);
}

int rsort_rccl_unique_id(void *id128) {
    if (!id128) return RSORT_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "NCCL_UNIQUE_ID_BYTES");
    return ncclGetUniqueId(static_cast<ncclUniqueId *>(id128)) == ncclSuccess ? RSORT_OK : RSORT_ERR_COMM;
}

int rsort_rccl_comm_init(void **comm, int world, int rank, const void *id128, int timeout_ms) {
    if (!comm || !id128 || world < 1 || rank < 0 || rank >= world) return RSORT_ERR_ARG;
    *comm = nullptr;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // returns at once; setup runs in the background and is polled below
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
    if (c == nullptr) return RSORT_ERR_COMM;
    comm_forget(c);  // (a new communicator at the address of one aborted earlier: this one is live)
    const int ms = timeout_ms > 0 ? timeout_ms : g_comm_timeout_ms.load();
    r = nb_complete(c, r, Clock::now() + std::chrono::milliseconds(ms));
    if (r != ncclSuccess) return comm_abort(c);  // (a peer never joined, or setup failed)
    *comm = c;
    return RSORT_OK;
}

int rsort_rccl_comm_destroy(void *comm) {
    if (!comm) return RSORT_ERR_ARG;
    if (comm_aborted((ncclComm_t)comm)) {  // released by the abort: only forget it
        comm_forget((ncclComm_t)comm);
        return RSORT_OK;
    }
    return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? RSORT_OK : RSORT_ERR_COMM;
}

int rsort_set_comm_timeout(int timeout_ms) {
    const int old = g_comm_timeout_ms.load();
    if (timeout_ms > 0) g_comm_timeout_ms.store(timeout_ms);
    return old;
}

int rsort_multi_inject_failure(int rank, int stage, int status) {
    if (rank < 0) {
        g_fail_rank.store(-1);
        g_fail_stage.store(0);
        return RSORT_OK;
    }
    if (stage < 1 || stage > 2 || status == RSORT_OK) return RSORT_ERR_ARG;
    g_fail_status.store(status);
    g_fail_stage.store(stage);
    g_fail_rank.store(rank);
    return RSORT_OK;
}

int rsort_multi_set_profiling(int enable) { return g_multi_prof.exchange(enable ? 1 : 0); }

int rsort_multi_last_stats(rsort_multi_stats *out) {
    if (!out || !t_stats_valid) return RSORT_ERR_ARG;
    *out = t_stats;
    return RSORT_OK;
}

int rsort_set_multi_options(int flags) {
    if ((flags & RSORT_MULTI_OVERLAP) && (flags & RSORT_MULTI_NO_OVERLAP)) return -RSORT_ERR_ARG;
    return g_multi_opts.exchange(flags & (RSORT_MULTI_OVERLAP | RSORT_MULTI_FULL | RSORT_MULTI_NO_OVERLAP));
}

int64_t rsort_set_exchange_piece(int64_t keys) {
    const int64_t old = g_piece.load();
    if (keys >= 64 && keys <= kMaxPiece) g_piece.store(keys);
    return old;
}

int rsort_host_transport_wrap(const rsort_host_transport *host, rsort_transport *out) {
    if (!host || !out || !host->allgather || !host->exchange || host->world < 1 || host->world > kMaxRanks ||
        host->rank < 0 || host->rank >= host->world)
        return RSORT_ERR_ARG;
    HostCtx *c = new (std::nothrow) HostCtx();
    if (!c) return RSORT_ERR_ALLOC;
    c->host = *host;
    *out = rsort_transport{c, host->world, host->rank, host_allgather, host_exchange};
    return RSORT_OK;
}

void rsort_host_transport_free(rsort_transport *wrapped) {
    if (!wrapped || wrapped->allgather != host_allgather) return;
    delete static_cast<HostCtx *>(wrapped->ctx);
    wrapped->ctx = nullptr;
}

int rsort_loopback_create(int world, void **group) {
    if (!group || world < 1 || world > kMaxRanks) return RSORT_ERR_ARG;
    LoopbackGroup *g = new (std::nothrow) LoopbackGroup();
    if (!g) return RSORT_ERR_ALLOC;
    g->world = world;
    for (int r = 0; r < world; ++r) g->ctx[r] = LoopbackCtx{g, r};
    *group = g;
    return RSORT_OK;
}

int rsort_loopback_transport(void *group, int rank, rsort_transport *out) {
    LoopbackGroup *g = static_cast<LoopbackGroup *>(group);
    if (!g || !out || rank < 0 || rank >= g->world) return RSORT_ERR_ARG;
    *out = rsort_transport{&g->ctx[rank], g->world, rank, lb_allgather, lb_exchange};
    return RSORT_OK;
}

void rsort_loopback_destroy(void *group) {
    delete static_cast<LoopbackGroup *>(group);
}

}  // extern "C"
