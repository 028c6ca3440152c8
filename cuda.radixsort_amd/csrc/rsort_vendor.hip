// rsort_vendor.hip -- the vendor comparator: rocPRIM's device radix sort.
//
// The reference's SORT_BY_THRUST branch (Parallel7.cu:69-73, thrust::sort on a
// device_vector) resolves on ROCm to rocThrust -> rocPRIM radix sort. It is reported next to
// our own sort as the "vendor ceiling" column; parity never depends on it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <rocprim/device/device_radix_sort.hpp>

#include "rsort.h"

namespace {
size_t vendor_temp_bytes(int64_t n) {
    size_t bytes = 0;
    if (rocprim::radix_sort_keys(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                 (size_t)n, 0, 32, (hipStream_t)0, false) != hipSuccess)
        return 0;
    return bytes;
}
}  // namespace

extern "C" {

size_t rsort_vendor_workspace_size(int64_t n) {
    if (n < 0) return 0;
    return vendor_temp_bytes(n > 0 ? n : 1) + 256;
}

int rsort_u32_vendor_device(const uint32_t *d_in, uint32_t *d_out, int64_t n, void *d_workspace,
                            size_t workspace_bytes, void *stream) {
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (n == 0) return RSORT_OK;
    if (!d_in || !d_out || !d_workspace) return RSORT_ERR_ARG;
    size_t bytes = vendor_temp_bytes(n);
    if (bytes == 0 || workspace_bytes < bytes) return RSORT_ERR_WORKSPACE;
    hipError_t e = rocprim::radix_sort_keys(d_workspace, bytes, d_in, d_out, (size_t)n, 0, 32,
                                            (hipStream_t)stream, false);
    return e == hipSuccess ? RSORT_OK : RSORT_ERR_HIP;
}

int rsort_u32_vendor(const uint32_t *in, uint32_t *out, int64_t n) {
    if (n < 0 || n >= ((int64_t)1 << 32)) return RSORT_ERR_SIZE;
    if (n == 0) return RSORT_OK;
    if (!in || !out) return RSORT_ERR_ARG;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return RSORT_ERR_NODEV;
    const size_t nb = ((size_t)n * 4 + 255) & ~(size_t)255;
    const size_t ws = rsort_vendor_workspace_size(n);
    void *buf = nullptr;
    if (hipMalloc(&buf, 2 * nb + ws) != hipSuccess) return RSORT_ERR_ALLOC;
    uint32_t *d_in = (uint32_t *)buf, *d_out = (uint32_t *)((char *)buf + nb);
    int st = RSORT_OK;
    if (hipMemcpy(d_in, in, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) st = RSORT_ERR_HIP;
    if (!st) st = rsort_u32_vendor_device(d_in, d_out, n, (char *)buf + 2 * nb, ws, nullptr);
    if (!st && hipMemcpy(out, d_out, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess)
        st = RSORT_ERR_HIP;
    (void)hipFree(buf);
    return st;
}

}  // extern "C"
