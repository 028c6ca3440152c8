// rsort_multi.cpp -- rsort_u32_multi: the multi-GPU sort over an RCCL communicator (C ABI).
//
// No reference counterpart (the reference sorts on one GPU, Parallel7.cu:10/:697); this is
// SURVEY.md §8e / BASELINE config 5, the same algorithm as cuda.radixsort_amd/multi.py (which
// drives it through torch.distributed): top-bits histogram, one all-reduce, splitters on bin
// edges, a stable partition into `world` key ranges, the count matrix by all-gather, ONE
// exchange (grouped send/recv: each pair of GPUs talks over its own xGMI link), a local sort.
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "rsort.h"
#include "rsort_internal.hpp"

using namespace rsort;

namespace {

constexpr int kTopBits = 12;
// splitters come from every 16th block of 256 keys: their balance only sets the load per rank
constexpr int kSampleStride = 16;
constexpr int kMaxRanks = kMaxSplitters + 1;
// keys per RCCL message piece (512 MiB): 1 GiB messages arrive whole, 2 GiB ones do not
constexpr unsigned long long kMaxMessage = 1ull << 27;

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct MultiCarve {
    uint32_t *part_k, *part_v, *hist32, *starts;
    unsigned long long *hist64, *sendc, *allc;
    void *sub;  // shared by the top histogram, the partition and the local sort (used in turn)
    size_t sub_bytes;
};

size_t sub_bytes(int64_t n, int64_t cap, int k, int pairs, int world) {
    size_t a = rsort_workspace_size(n, kTopBits, 0);
    size_t b = rsort_partition_workspace_size(n, world, pairs);
    // the received count is only known later; a smaller n can pick a geometry with a larger
    // chunk table (<= 2^k x 4096 entries), so leave room for that
    size_t c = rsort_workspace_size(std::max<int64_t>(cap, 1), k, pairs) + ((size_t)4 << k << 12);
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
    m.part_k = (uint32_t *)take((size_t)n * 4);
    m.part_v = pairs ? (uint32_t *)take((size_t)n * 4) : nullptr;
    m.hist32 = (uint32_t *)take((size_t)(1 << kTopBits) * 4);
    m.hist64 = (unsigned long long *)take((size_t)(1 << kTopBits) * 8);
    m.starts = (uint32_t *)take((size_t)(kMaxRanks + 1) * 4);
    m.sendc = (unsigned long long *)take((size_t)kMaxRanks * 8);
    m.allc = (unsigned long long *)take((size_t)kMaxRanks * kMaxRanks * 8);
    m.sub_bytes = sub_bytes(n, cap, k, pairs, world);
    m.sub = take(m.sub_bytes);
    if (mc) *mc = m;
    return off;
}

// world-1 ascending splitters on bin edges of the global top-bits histogram: bucket i ends with
// the first bin whose inclusive prefix reaches (i+1)*total/world (multi.py:choose_splitters).
std::vector<uint32_t> choose_splitters(const std::vector<unsigned long long> &hist, int world) {
    std::vector<unsigned long long> cum(hist.size());
    unsigned long long acc = 0;
    for (size_t i = 0; i < hist.size(); ++i) cum[i] = (acc += hist[i]);
    const unsigned long long total = acc;
    const int shift = 32 - kTopBits;
    std::vector<uint32_t> out;
    for (int i = 1; i < world; ++i) {
        const unsigned long long target = (total * (unsigned long long)i) / (unsigned long long)world;
        const size_t b = (size_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        const size_t edge = b + 1;
        uint32_t sp = edge < hist.size() ? (uint32_t)(edge << shift) : 0xFFFFFFFFu;
        if (!out.empty()) sp = std::max(sp, out.back());
        out.push_back(sp);
    }
    return out;
}

int nccl_status(ncclResult_t r) { return r == ncclSuccess ? RSORT_OK : RSORT_ERR_COMM; }

}  // namespace

extern "C" {

size_t rsort_multi_workspace_size(int64_t n, int64_t capacity, int k_bits, int pairs, int world) {
    if (n < 0 || capacity < 0 || world < 1 || world > kMaxRanks) return 0;
    return multi_bytes(n, capacity, k_bits, pairs ? 1 : 0, world, nullptr, nullptr);
}

int rsort_u32_multi(const uint32_t *d_keys, const uint32_t *d_vals, int64_t n, uint32_t *d_keys_out,
                    uint32_t *d_vals_out, int64_t capacity, int64_t *out_n, int64_t *out_offset, int k_bits,
                    void *nccl_comm, void *d_workspace, size_t workspace_bytes, void *stream) {
    if (k_bits < kMinBits || k_bits > kMaxBits) return RSORT_ERR_BITS;
    if (n < 0 || n >= ((int64_t)1 << 32) || capacity < 0 || capacity >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (!nccl_comm || !out_n || !out_offset || !d_workspace) return RSORT_ERR_ARG;
    const int pairs = d_vals != nullptr;
    if ((n > 0 && !d_keys) || (capacity > 0 && (!d_keys_out || (pairs && !d_vals_out)))) return RSORT_ERR_ARG;
    ncclComm_t comm = (ncclComm_t)nccl_comm;
    int world = 0, me = 0;
    if (ncclCommCount(comm, &world) != ncclSuccess || ncclCommUserRank(comm, &me) != ncclSuccess)
        return RSORT_ERR_COMM;
    if (world < 1 || world > kMaxRanks) return RSORT_ERR_ARG;
    MultiCarve m;
    if (workspace_bytes < multi_bytes(n, capacity, k_bits, pairs, world, &m, d_workspace)) return RSORT_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    int st;

    // 1-3: global top-bits histogram -> splitters (host)
    if ((st = rsort_top_histogram_sampled(d_keys, n, kTopBits, kSampleStride, m.hist32, stream))) return st;
    if (launch_widen(m.hist32, m.hist64, 1u << kTopBits, s) != hipSuccess) return RSORT_ERR_HIP;
    if ((st = nccl_status(ncclAllReduce(m.hist64, m.hist64, (size_t)1 << kTopBits, ncclUint64, ncclSum, comm, s))))
        return st;
    std::vector<unsigned long long> hist((size_t)1 << kTopBits);
    if (hipMemcpyAsync(hist.data(), m.hist64, hist.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return RSORT_ERR_HIP;
    const std::vector<uint32_t> split = choose_splitters(hist, world);

    // 4: stable partition of the local keys into `world` key ranges
    if ((st = rsort_partition_device(d_keys, d_vals, m.part_k, m.part_v, n, split.data(), world, m.starts, m.sub,
                                     m.sub_bytes, stream)))
        return st;
    uint32_t starts[kMaxRanks + 1];
    if (hipMemcpyAsync(starts, m.starts, (size_t)(world + 1) * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return RSORT_ERR_HIP;
    unsigned long long send[kMaxRanks];
    for (int r = 0; r < world; ++r) send[r] = (unsigned long long)(starts[r + 1] - starts[r]);

    // 5: the world x world count matrix (row = source rank)
    if (hipMemcpyAsync(m.sendc, send, (size_t)world * 8, hipMemcpyHostToDevice, s) != hipSuccess) return RSORT_ERR_HIP;
    if ((st = nccl_status(ncclAllGather(m.sendc, m.allc, (size_t)world, ncclUint64, comm, s)))) return st;
    unsigned long long all[kMaxRanks * kMaxRanks];
    if (hipMemcpyAsync(all, m.allc, (size_t)world * world * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return RSORT_ERR_HIP;
    unsigned long long recv[kMaxRanks], n_recv = 0, offset = 0;
    for (int r = 0; r < world; ++r) {
        recv[r] = all[r * world + me];
        n_recv += recv[r];
        for (int q = 0; q < me; ++q) offset += all[r * world + q];
    }
    if (n_recv > (unsigned long long)capacity) return RSORT_ERR_CAPACITY;

    // 6: the exchange; chunks land in source-rank order (keeps pairs stable). Every message is
    // cut into pieces of at most kMaxMessage keys: this RCCL (2.26, ROCm 7) silently leaves the
    // second half of a >= 2 GiB message unwritten (dev/a2a_lab.py), and with 2^30 keys per GPU
    // two ranks exchange ~2 GiB each way. The piece count comes from the whole count matrix, so
    // every rank runs the same number of groups.
    unsigned long long biggest = 0;
    for (int i = 0; i < world * world; ++i) biggest = std::max(biggest, all[i]);
    const unsigned long long pieces = std::max(1ull, (biggest + kMaxMessage - 1) / kMaxMessage);
    for (unsigned long long q = 0; q < pieces; ++q) {
        if ((st = nccl_status(ncclGroupStart()))) return st;
        unsigned long long so = 0, ro = 0;
        for (int r = 0; r < world; ++r) {
            const unsigned long long a0 = std::min(send[r], q * kMaxMessage), a1 = std::min(send[r], (q + 1) * kMaxMessage);
            const unsigned long long b0 = std::min(recv[r], q * kMaxMessage), b1 = std::min(recv[r], (q + 1) * kMaxMessage);
            if (a1 > a0) {
                ncclSend(m.part_k + so + a0, a1 - a0, ncclUint32, r, comm, s);
                if (pairs) ncclSend(m.part_v + so + a0, a1 - a0, ncclUint32, r, comm, s);
            }
            if (b1 > b0) {
                ncclRecv(d_keys_out + ro + b0, b1 - b0, ncclUint32, r, comm, s);
                if (pairs) ncclRecv(d_vals_out + ro + b0, b1 - b0, ncclUint32, r, comm, s);
            }
            so += send[r];
            ro += recv[r];
        }
        if ((st = nccl_status(ncclGroupEnd()))) return st;
    }

    // 7: local sort of what arrived, in place
    if (n_recv > 0) {
        rsort_plan p;
        if ((st = rsort_plan_make((int64_t)n_recv, k_bits, pairs, 0, &p))) return st;
        if ((st = rsort_sort_planned(&p, d_keys_out, d_vals_out, d_keys_out, d_vals_out, m.sub, m.sub_bytes, stream)))
            return st;
    }
    *out_n = (int64_t)n_recv;
    *out_offset = (int64_t)offset;
    return RSORT_OK;
}

}  // extern "C"
