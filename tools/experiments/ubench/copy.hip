// Stream-copy bandwidth sweep (diagnostic, not the product): the 16-B-per-lane copy of
// flodbadd_amd/csrc/fb_bwref.hip over 1 GiB at several grid sizes / units per thread, with plain
// and nontemporal loads and stores.  Prints GB/s (read + written bytes).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n16) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n16) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

template <int U, bool NT>
static void run(u32x4* d, const u32x4* s, size_t n16, unsigned grid) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_copy<U, NT>), dim3(grid), dim3(256), 0, nullptr, d, s, n16);
    (void)hipEventRecord(a, nullptr);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copy<U, NT>), dim3(grid), dim3(256), 0, nullptr, d, s, n16);
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("U=%d NT=%d grid=%u  %.1f GB/s\n", U, (int)NT, grid, 2.0 * n16 * 16.0 * reps / (ms / 1e3) / 1e9);
    fflush(stdout);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main() {
    const size_t bytes = 1ull << 30, n16 = bytes / 16;
    u32x4 *s = nullptr, *d = nullptr;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMemset(s, 1, bytes);
    (void)hipDeviceSynchronize();
    for (unsigned mult : {2u, 4u, 8u, 16u, 64u}) {
        const unsigned grid = 256u * mult;
        run<1, false>(d, s, n16, grid);
        run<4, false>(d, s, n16, grid);
        run<8, false>(d, s, n16, grid);
        run<4, true>(d, s, n16, grid);
        run<8, true>(d, s, n16, grid);
    }
    const unsigned full = (unsigned)(n16 / 256);  // one unit per thread, no loop
    run<1, false>(d, s, n16, full);
    run<1, true>(d, s, n16, full);
    (void)hipFree(s);
    (void)hipFree(d);
    return 0;
}
