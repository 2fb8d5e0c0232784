// fb_bwref.hip -- the stream-copy bandwidth reference of bench.py ("also report
// the fraction of measured stream-copy BW").  Not part of the product path or its C ABI: a plain
// 16-B-per-lane copy (the float4 copy MI355X_MICROARCH.md measures at ~6.3 TB/s), built into its
// own library, libfb_bwref.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kThreads = 256;
constexpr int kUnroll = 4;  // 16-B units per thread and step, all loads in flight before the stores
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kThreads) void k_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * kThreads * kUnroll;
    for (size_t base = (size_t)blockIdx.x * kThreads * kUnroll + threadIdx.x; base < n16; base += stride) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const size_t i = base + (size_t)u * kThreads;
            if (i < n16) v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const size_t i = base + (size_t)u * kThreads;
            if (i < n16) dst[i] = v[u];
        }
    }
}
}  // namespace

// Copies `bytes` (a multiple of 16) from src to dst `reps` times on the null stream after two
// untimed copies; *ms = the events' elapsed time of the timed copies.  Returns a hipError_t.
extern "C" int fb_bwref_copy(void* dst, const void* src, size_t bytes, int reps, float* ms) {
    if (!dst || !src || !ms || reps <= 0 || (bytes & 15u)) return (int)hipErrorInvalidValue;
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int)e;
    const size_t n16 = bytes / 16u;
    const unsigned grid = (unsigned)cus * 8u;
    hipEvent_t a = nullptr, b = nullptr;
    if ((e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess) return (int)e;
    for (int r = 0; r < 2; ++r)
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(kThreads), 0, nullptr, (u32x4*)dst, (const u32x4*)src, n16);
    (void)hipEventRecord(a, nullptr);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(kThreads), 0, nullptr, (u32x4*)dst, (const u32x4*)src, n16);
    (void)hipEventRecord(b, nullptr);
    e = hipEventSynchronize(b);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventElapsedTime(ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return (int)e;
}
