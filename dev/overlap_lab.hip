// Backs DESIGN §5 "Overlap on one GPU" (round 6): what RSORT_MULTI_OVERLAP's lower-half
// sort costs when the exchange's kernels share the CUs. RCCL's point-to-point kernels stay resident for the
// whole exchange (one workgroup per channel, looping over the message at the xGMI link rate), so the
// stand-in here is a copy kernel that holds `wgs` workgroups of 256 threads for as long as a paced copy of
// `bytes` at `gbps` takes: it reads and writes HBM at that rate (as the exchange reads its send buffer
// and receives its peers' writes) and occupies the CUs its workgroups land on.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC dev/overlap_lab.hip -o dev/liboverlap_lab.so
//   (loaded by dev/multi_model.py through ctypes; nothing of the library links it)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Workgroup b copies its share [b * share, (b + 1) * share) of the quads, 4 quads per thread per step,
// and after each step waits (s_sleep) until the steady counter (wall_clock64, hipDeviceAttributeWallClockRate) reaches its pace: share bytes
// spread evenly over bytes / gbps. gbps <= 0: no pacing (a plain copy at the rate the CUs get).
__global__ __launch_bounds__(256) void hold_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                 uint64_t quads, double ticks_per_quad) {
    const uint64_t share = (quads + gridDim.x - 1) / gridDim.x;
    const uint64_t beg = (uint64_t)blockIdx.x * share;
    const uint64_t end = beg + share < quads ? beg + share : quads;
    const uint64_t t0 = (uint64_t)wall_clock64();
    for (uint64_t q = beg; q < end; q += 4 * 256) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = q + threadIdx.x + j * 256;
            if (i < end) v[j] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = q + threadIdx.x + j * 256;
            if (i < end) __builtin_nontemporal_store(v[j], dst + i);
        }
        if (ticks_per_quad > 0.0) {
            const uint64_t due = t0 + (uint64_t)((double)(q + 4 * 256 - beg) * ticks_per_quad);
            while ((uint64_t)wall_clock64() < due) __builtin_amdgcn_s_sleep(32);
        }
    }
}

extern "C" __attribute__((visibility("default"))) int lab_hold(const void *src, void *dst, uint64_t bytes, int wgs,
                                                               double gbps, void *stream) {
    if (wgs <= 0 || bytes < 16) return 1;
    const uint64_t quads = bytes / 16;
    // each workgroup moves quads / wgs at gbps / wgs; the steady counter's rate from the device
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        return 6;
    const double ticks = gbps > 0.0 ? (double)khz * 1e3 * 16.0 * (double)wgs / (gbps * 1e9) : 0.0;
    hold_copy<<<wgs, 256, 0, (hipStream_t)stream>>>((const u32x4 *)src, (u32x4 *)dst, quads, ticks);
    return hipGetLastError() == hipSuccess ? 0 : 6;
}
