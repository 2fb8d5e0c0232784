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

// The k_parse_seg access shape without the parse: one wave per 64-frame segment (each lane
// gathers its 64-B frame as four 16-B loads), the segment's 3.5 KiB of records written as
// coalesced 16-B stores (14 of each 16-uint4 block).  kPersist: 768 blocks x 8 waves, block-
// interleaved segments handed out inside the block from an LDS counter (the product mapping);
// else one short block per 8 x kSegsPerWave segments (the hardware dispatcher balances).
template <bool kPersist, int kSegsPerWave>
__global__ __launch_bounds__(512) void k_segcopy(Pairs p, uint32_t nb, size_t n16) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __shared__ uint32_t s_next;
    const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t segs_per_batch = (uint32_t)(n16 / 256u);  // 4 KiB of input per segment
    const uint32_t nseg = nb * segs_per_batch;
    if (threadIdx.x == 0) s_next = 8u;
    __syncthreads();
    uint32_t L = wave;
    for (int it = 0;; ++it) {
        uint32_t sg;
        if (kPersist) sg = blockIdx.x * 8u + L % 8u + (L / 8u) * (gridDim.x * 8u);
        else sg = (blockIdx.x * 8u + wave) * kSegsPerWave + it;
        if (!kPersist && it >= kSegsPerWave) break;
        if (sg >= nseg) break;
        const uint32_t b = sg / segs_per_batch, ls = sg - b * segs_per_batch;
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)p.in[b], 0, (int)(n16 * 16), 0x00020000);
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)p.out[b], 0, (int)(n16 / 16 * 14 * 16), 0x00020000);
        const uint32_t fo = ls * 4096u + lane * 64u;
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(ri, fo, 0, 0);
        const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(ri, fo + 16u, 0, 0);
        const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(ri, fo + 32u, 0, 0);
        const u32x4 e = __builtin_amdgcn_raw_buffer_load_b128(ri, fo + 48u, 0, 0);
        const u32x4 x = a ^ c ^ d ^ e;
        const uint32_t oo = ls * 3584u;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < 3 || lane < 32u) __builtin_amdgcn_raw_buffer_store_b128(x, ro, oo + (k * 64u + lane) * 16u, 0, 2);
        if (kPersist) {
            uint32_t v = 0u;
            if (lane == 0u) v = atomicAdd(&s_next, 1u);
            L = __builtin_amdgcn_readfirstlane(v);
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
    {
        const uint32_t nseg = nb * (uint32_t)(n16 / 256u);
        const int shapes = 4;
        const char* names[shapes] = {"seg persist 768x8w", "seg short 8/wave", "seg short 2/wave", "seg short 32/wave"};
        for (int v = 0; v < shapes; ++v) {
            float best = 1e30f;
            for (int it = -2; it < iters; ++it) {
                CK(hipEventRecord(e0, 0));
                if (v == 0) hipLaunchKernelGGL((k_segcopy<true, 1>), dim3(768), dim3(512), 0, 0, p, nb, n16);
                else if (v == 1) hipLaunchKernelGGL((k_segcopy<false, 8>), dim3((nseg + 63) / 64), dim3(512), 0, 0, p, nb, n16);
                else if (v == 2) hipLaunchKernelGGL((k_segcopy<false, 2>), dim3((nseg + 15) / 16), dim3(512), 0, 0, p, nb, n16);
                else hipLaunchKernelGGL((k_segcopy<false, 32>), dim3((nseg + 255) / 256), dim3(512), 0, 0, p, nb, n16);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 0 && ms < best) best = ms;
            }
            printf("{\"shape\": \"%s\", \"batches\": %u, \"ms\": %.4f, \"TBs\": %.3f, \"us_per_batch\": %.2f}\n", names[v], nb, best,
                   bytes / (best * 1e9), best * 1e3 / nb);
        }
    }
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
