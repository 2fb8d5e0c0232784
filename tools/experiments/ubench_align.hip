// Microbenchmark: header-window loads of 64-B frames at 2-mod-4 byte offsets (10, 26, 42 + a dword
// at 66, as k_parse_seg issues them) vs dword-aligned ones (8, 24, 40 + 64), one lane per frame,
// each lane storing 56 B (as a record) so the read/write mix matches C2.
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/ubench_align tools/experiments/ubench_align.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int OFF>
__global__ __launch_bounds__(512) void k_win(const uint8_t* __restrict__ f, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)f, (short)0, (int)(n * 64u), 0x00020000);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t o0 = i * 64u + OFF;
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, o0, 0, 0);
        const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, o0 + 16u, 0, 0);
        const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(r, o0 + 32u, 0, 0);
        const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(r, o0 + 56u, 0, 0);
        uint32_t* o = out + (size_t)i * 14u;
        const uint32_t x = a.x ^ b.y ^ c.z ^ d;
        *reinterpret_cast<uint2*>(o) = make_uint2(a.y ^ x, a.z);
        *reinterpret_cast<uint4*>(o + 2) = make_uint4(a.w, b.x, b.z, b.w);
        *reinterpret_cast<uint4*>(o + 6) = make_uint4(c.x, c.y, c.w, x);
        *reinterpret_cast<uint4*>(o + 10) = make_uint4(a.x, b.y, c.z, d);
    }
}

template <int OFF>
static float run(const uint8_t* f, uint32_t n, uint32_t* out, int reps) {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint32_t grid = (uint32_t)cus * 4u;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_win<OFF>, dim3(grid), dim3(512), 0, 0, f, n, out);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_win<OFF>, dim3(grid), dim3(512), 0, 0, f, n, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const uint32_t n = 8u << 20;  // 8M frames: 512 MiB in, 448 MiB out
    uint8_t* f;
    uint32_t* out;
    CK(hipMalloc(&f, (size_t)n * 64u + 256u));
    CK(hipMalloc(&out, (size_t)n * 56u));
    CK(hipMemset(f, 1, (size_t)n * 64u + 256u));
    for (int round = 0; round < 3; ++round) {
        const float t10 = run<10>(f, n, out, 20), t8 = run<8>(f, n, out, 20), t12 = run<12>(f, n, out, 20);
        const double bytes = (double)n * (64.0 + 56.0);
        printf("round %d  off10 %.1f us %.0f GB/s | off8 %.1f us %.0f GB/s | off12 %.1f us %.0f GB/s\n", round,
               t10 * 1e3, bytes / t10 / 1e6, t8 * 1e3, bytes / t8 / 1e6, t12 * 1e3, bytes / t12 / 1e6);
    }
    CK(hipFree(f));
    CK(hipFree(out));
    return 0;
}
