// LDS atomic / cross-lane reduction microbenchmark (diagnostic, not the product).  K1c and K2 apply
// each record with ~10 LDS atomics; under skewed popularity a wave's lanes mostly hit ONE slot.  This
// measures, with four 256-thread workgroups per CU on every CU (K1c's geometry), the CU cycles per
// wave instruction of:
//   same     ds_add_u32, all 64 lanes one address          distinct  ds_add_u32, 64 addresses
//   same64   ds_add_u64, all 64 lanes one address          min       ds_min_u32, one address
//   bperm    a 6-step __shfl_xor (ds_bpermute) sum reduction, per reduction
//   dpp      a 6-step DPP sum reduction to lane 63 (quad_perm, row_half_mirror, row_mirror,
//            row_bcast15 / 31) + readlane, per reduction
// Build: hipcc -O3 --offload-arch=gfx950 -o ldsatom ldsatom.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kIters = 2048;

__device__ __forceinline__ uint32_t dpp_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false); // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false); // row_mirror
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast31 -> rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
    __shared__ unsigned long long lds[2048];
    for (uint32_t i = threadIdx.x; i < 2048u; i += 256u) lds[i] = 0ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t* l32 = reinterpret_cast<uint32_t*>(lds);
    uint32_t acc = seed + lane;
    for (int it = 0; it < kIters; ++it) {
        if (MODE == 0) atomicAdd(l32 + wave * 64u, acc);
        if (MODE == 1) atomicAdd(l32 + wave * 64u + lane, acc);
        if (MODE == 2) atomicAdd(lds + wave * 32u, (unsigned long long)acc);
        if (MODE == 3) atomicMin(l32 + wave * 64u, acc + (uint32_t)it);
        if (MODE == 4) {
            uint32_t v = acc + (uint32_t)it;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            acc ^= v;
        }
        if (MODE == 5) acc ^= dpp_sum(acc + (uint32_t)it);
    }
    __syncthreads();
    out[blockIdx.x * 256u + threadIdx.x] = acc + l32[threadIdx.x];
}

__global__ void kcheck(uint32_t* out) {
    out[threadIdx.x] = dpp_sum(threadIdx.x * 3u + 1u);  // sum over 64 lanes = 3 * 2016 + 64 = 6112
}

template <int MODE>
static void run(const char* name, uint32_t* d, int grid, int cus, float clk_ghz) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, d, 1u);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, d, (uint32_t)r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double waves_per_cu = (double)grid * 4.0 / cus;
    const double cyc = ms / 5.0 * 1e-3 * clk_ghz * 1e9;
    printf("%-9s %8.3f ms/launch  %7.2f CU cycles per wave-instruction (per reduction for bperm/dpp)\n", name,
           ms / 5.0, cyc / (waves_per_cu * kIters));
}

int main() {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    const float clk = pr.clockRate / 1e6f;  // kHz -> GHz
    const int grid = cus * 4;
    uint32_t* d;
    CK(hipMalloc(&d, (size_t)grid * 256 * 4));
    printf("CUs %d, clock %.2f GHz, %d workgroups of 256 threads, %d iterations\n", cus, clk, grid, kIters);
    run<0>("same", d, grid, cus, clk);
    run<1>("distinct", d, grid, cus, clk);
    run<2>("same64", d, grid, cus, clk);
    run<3>("min", d, grid, cus, clk);
    run<4>("bperm", d, grid, cus, clk);
    run<5>("dpp", d, grid, cus, clk);
    hipLaunchKernelGGL(kcheck, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[64];
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 64; ++i) bad += h[i] != 6112u;
    printf("dpp_sum check: %s (lane 0 got %u, expected 6112)\n", bad ? "FAIL" : "ok", h[0]);
    CK(hipFree(d));
    return 0;
}
