// fb_bwref.hip -- the stream-copy bandwidth reference of bench.py ("also report
// the fraction of measured stream-copy BW").  Not part of the product path or its C ABI: a plain
// 16-B-per-lane copy, built into its own library, libfb_bwref.so.  Shape from the sweep in
// tools/experiments/ubench/copy.hip (profiles/r04_ubench_copy.txt, 1 GiB): one 16-B unit per
// thread and no loop, nontemporal loads and stores, 6.52 TB/s; grid-stride loops of 1-8 units
// per thread at 512-16,384 workgroups 4.6-6.1 TB/s; hipMemcpyAsync device to device ~4.7 TB/s.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
}  // namespace

// Copies `bytes` (a multiple of 16, at most 2^42) from src to dst `reps` times on the null stream
// after two untimed copies; *ms = the events' elapsed time of the timed copies.  Returns a hipError_t.
extern "C" int fb_bwref_copy(void* dst, const void* src, size_t bytes, int reps, float* ms) {
    if (!dst || !src || !ms || reps <= 0 || (bytes & 15u) || bytes == 0 || bytes > (1ull << 42))
        return (int)hipErrorInvalidValue;
    const size_t n16 = bytes / 16u;
    const unsigned grid = (unsigned)((n16 + 255u) / 256u);
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e;
    if ((e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess) return (int)e;
    for (int r = 0; r < 2; ++r)
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, nullptr, (u32x4*)dst, (const u32x4*)src, n16);
    (void)hipEventRecord(a, nullptr);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, nullptr, (u32x4*)dst, (const u32x4*)src, n16);
    (void)hipEventRecord(b, nullptr);
    e = hipEventSynchronize(b);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventElapsedTime(ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return (int)e;
}
