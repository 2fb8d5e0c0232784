// ubench_copy.hip -- streaming ceiling for the C2 access mix (not product code).
// 32 batch pairs of (64 MiB read, 56 MiB written: the C2 frames and records) streamed by ONE
// launch, like one 32-batch k_parse_seg launch; reports TB/s of read + written bytes for a few
// launch shapes and store policies.  Usage: ubench_copy [batches=32] [iters=20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

struct Pairs {
    const uint4* in[32];
    uint4* out[32];
};

// Each 64-B frame-equivalent: 4 x 16-B reads; each 56-B record equivalent: 3.5 x 16-B writes
// (written as 7 x 8-B halves would be odd; instead 14 of every 16 input uint4 are written).
template <int kAux>
__global__ __launch_bounds__(256) void k_mix(Pairs p, uint32_t nb, size_t n16) {
    const size_t total = (size_t)nb * n16;
    for (size_t g = blockIdx.x * 256ull + threadIdx.x; g < total; g += (size_t)gridDim.x * 256ull) {
        const uint32_t b = __builtin_amdgcn_readfirstlane((uint32_t)(g >> 22));  // n16 = 2^22 (64 MiB per batch); wave-uniform
        const size_t i = g & ((1ull << 22) - 1);
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)p.in[b], 0, (int)(n16 * 16), 0x00020000);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(i * 16), 0, 0);
        const size_t o = (i >> 4) * 14 + (i & 15);  // 14 of 16
        if ((i & 15) < 14) {
            const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)p.out[b], 0, (int)(n16 / 16 * 14 * 16), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, (uint32_t)(o * 16), 0, kAux);
        }
    }
}

// 4 loads in flight per lane before their stores.
template <int kAux>
__global__ __launch_bounds__(256) void k_mix4(Pairs p, uint32_t nb, size_t n16) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const size_t total = (size_t)nb * n16, stride = (size_t)gridDim.x * 256ull;
    for (size_t g0 = blockIdx.x * 256ull + threadIdx.x; g0 < total; g0 += 4 * stride) {
        u32x4 v[4];
        uint32_t bb[4];
        size_t ii[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t g = g0 + u * stride;
            bb[u] = __builtin_amdgcn_readfirstlane((uint32_t)(min(g, total - 1) >> 22));
            ii[u] = g & ((1ull << 22) - 1);
            const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)p.in[bb[u]], 0, (int)(n16 * 16), 0x00020000);
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, g < total ? (uint32_t)(ii[u] * 16) : 0xFFFFFFF0u, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t g = g0 + u * stride;
            const size_t i = ii[u], o = (i >> 4) * 14 + (i & 15);
            if (g < total && (i & 15) < 14) {
                const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)p.out[bb[u]], 0, (int)(n16 / 16 * 14 * 16), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(v[u], ro, (uint32_t)(o * 16), 0, kAux);
            }
        }
    }
}

// Each block streams its own contiguous range (the k_parse_seg mapping: block-owned ranges).
template <int kAux>
__global__ __launch_bounds__(256) void k_mix_range(Pairs p, uint32_t nb, size_t n16) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const size_t total = (size_t)nb * n16, per = (total / gridDim.x + 255) & ~255ull;
    const size_t lo = blockIdx.x * per, hi = min(total, lo + per);
    for (size_t g = lo + threadIdx.x; g < hi; g += 256) {
        const uint32_t b = __builtin_amdgcn_readfirstlane((uint32_t)(g >> 22));
        const size_t i = g & ((1ull << 22) - 1);
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)p.in[b], 0, (int)(n16 * 16), 0x00020000);
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(i * 16), 0, 0);
        const size_t o = (i >> 4) * 14 + (i & 15);
        if ((i & 15) < 14) {
            const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)p.out[b], 0, (int)(n16 / 16 * 14 * 16), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, (uint32_t)(o * 16), 0, kAux);
        }
    }
}

int main(int argc, char** argv) {
    const uint32_t nb = argc > 1 ? (uint32_t)atoi(argv[1]) : 32u;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const size_t in_bytes = 64ull << 20, n16 = in_bytes / 16, out_bytes = n16 / 16 * 14 * 16;
    Pairs p;
    for (uint32_t b = 0; b < nb; ++b) {
        CK(hipMalloc((void**)&p.in[b], in_bytes));
        CK(hipMalloc((void**)&p.out[b], out_bytes));
        CK(hipMemset((void*)p.in[b], b, in_bytes));
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)nb * (in_bytes + out_bytes);
    const int grids[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536};
    for (int aux = 0; aux < 5; ++aux) {
        for (int gi = 0; gi < 7; ++gi) {
            const int grid = grids[gi];
            float best = 1e30f;
            for (int it = -2; it < iters; ++it) {
                CK(hipEventRecord(e0, 0));
                if (aux == 1) hipLaunchKernelGGL(k_mix<2>, dim3(grid), dim3(256), 0, 0, p, nb, n16);
                else if (aux == 0) hipLaunchKernelGGL(k_mix<0>, dim3(grid), dim3(256), 0, 0, p, nb, n16);
                else if (aux == 2) hipLaunchKernelGGL(k_mix4<0>, dim3(grid), dim3(256), 0, 0, p, nb, n16);
                else if (aux == 3) hipLaunchKernelGGL(k_mix4<2>, dim3(grid), dim3(256), 0, 0, p, nb, n16);
                else hipLaunchKernelGGL(k_mix_range<2>, dim3(grid), dim3(256), 0, 0, p, nb, n16);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 0 && ms < best) best = ms;
            }
            printf("{\"store\": \"%s\", \"grid\": %d, \"batches\": %u, \"ms\": %.4f, \"TBs\": %.3f, \"us_per_batch\": %.2f}\n",
                   aux == 4 ? "range nt" : (aux & 1) ? (aux > 1 ? "x4 nt" : "nt") : (aux > 1 ? "x4 default" : "default"), grid, nb, best, bytes / (best * 1e9), best * 1e3 / nb);
        }
    }
    return 0;
}
