// ubench_gather.hip -- random record gathers on MI355X (not product code).
// One lane per record: record idx[i] (56-B or 64-B stride) is loaded and folded into out[i].
// Reports G records/s for: identity order (streaming), a random permutation over the whole buffer
// (the table update's gather pattern), and the same over a buffer small enough for the Infinity
// Cache.  Usage: ubench_gather [records=10485760] [reps=10]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <uint32_t kStride, int kPer>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* buf, uint64_t bytes, const uint32_t* idx, uint32_t n,
                                                uint32_t* out) {
    // kPer records per lane, all loads issued before any use (flat loads: the product's ld_u4)
    const uint32_t i0 = (blockIdx.x * 256u + threadIdx.x) * kPer;
    if (i0 >= n) return;
    uint4 v[kPer][4];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t* r = reinterpret_cast<const uint32_t*>(buf + (uint64_t)idx[min(i0 + k, n - 1)] * kStride);
        __builtin_memcpy(&v[k][0], r, 16);
        __builtin_memcpy(&v[k][1], r + 4, 16);
        __builtin_memcpy(&v[k][2], r + 8, 16);
        if (kStride == 64) __builtin_memcpy(&v[k][3], r + 12, 16);
        else { __builtin_memcpy(&v[k][3], r + 12, 8); v[k][3].z = v[k][3].w = 0u; }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x ^= v[k][j].x ^ v[k][j].y ^ v[k][j].z ^ v[k][j].w;
        if (i0 + k < n) out[i0 + k] = x;
    }
}

// Runs of `run` consecutive 64-B entries starting at random run positions (the read pattern of a
// partition-bucketed entry array): lane i reads entry base[i / run] + i % run.
__global__ __launch_bounds__(256) void k_runs(const uint4* ent, const uint32_t* base, uint32_t run, uint32_t n,
                                              uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint4* e = ent + (size_t)(base[i / run] + i % run) * 4u;
    const uint4 a = e[0], b = e[1], c = e[2], d = e[3];
    out[i] = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ d.x;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t splitmix() {
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 10485760u;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    std::vector<uint32_t> perm(N), ident(N);
    for (uint32_t i = 0; i < N; ++i) perm[i] = ident[i] = i;
    for (uint32_t i = N - 1; i > 0; --i) std::swap(perm[i], perm[splitmix() % (i + 1)]);
    uint8_t* buf;
    uint32_t *d_perm, *d_ident, *d_out, *d_small;
    const uint64_t bytes = (uint64_t)N * 64u;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    CK(hipMalloc(&d_perm, N * 4ull));
    CK(hipMalloc(&d_ident, N * 4ull));
    CK(hipMalloc(&d_out, N * 4ull));
    CK(hipMalloc(&d_small, N * 4ull));
    CK(hipMemcpy(d_perm, perm.data(), N * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ident, ident.data(), N * 4ull, hipMemcpyHostToDevice));
    // a permutation confined to the first M records (an Infinity-Cache-sized buffer), N lanes
    const uint32_t M = 1u << 21;
    std::vector<uint32_t> small(N);
    for (uint32_t i = 0; i < N; ++i) small[i] = (uint32_t)(splitmix() % M);
    CK(hipMemcpy(d_small, small.data(), N * 4ull, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t grid = (N + 255) / 256;
    auto timeit = [&](const char* name, auto launch, double bytes_per) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("%-40s %9.1f us  %7.2f G rec/s  %7.2f TB/s of records\n", name, us, N / us / 1e3,
               N * bytes_per / us / 1e6);
    };
    timeit("56B identity", [&] { hipLaunchKernelGGL((k_gather<56, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_ident, N, d_out); }, 56);
    timeit("56B random (N x 56 B buffer)", [&] { hipLaunchKernelGGL((k_gather<56, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_perm, N, d_out); }, 56);
    timeit("56B random, 2 per lane", [&] { hipLaunchKernelGGL((k_gather<56, 2>), dim3((grid + 1) / 2), dim3(256), 0, 0, buf, bytes, d_perm, N, d_out); }, 56);
    timeit("56B random, 4 per lane", [&] { hipLaunchKernelGGL((k_gather<56, 4>), dim3((grid + 3) / 4), dim3(256), 0, 0, buf, bytes, d_perm, N, d_out); }, 56);
    timeit("64B identity", [&] { hipLaunchKernelGGL((k_gather<64, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_ident, N, d_out); }, 64);
    timeit("64B random (N x 64 B buffer)", [&] { hipLaunchKernelGGL((k_gather<64, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_perm, N, d_out); }, 64);
    timeit("56B random within 2M records (112 MB)", [&] { hipLaunchKernelGGL((k_gather<56, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_small, N, d_out); }, 56);
    timeit("64B random within 2M records (128 MB)", [&] { hipLaunchKernelGGL((k_gather<64, 1>), dim3(grid), dim3(256), 0, 0, buf, bytes, d_small, N, d_out); }, 64);
    for (uint32_t run : {2u, 5u, 8u, 16u, 32u}) {
        const uint32_t nr = N / run;
        std::vector<uint32_t> base(nr);
        for (uint32_t k = 0; k < nr; ++k) base[k] = (uint32_t)(splitmix() % (N / run)) * run;
        uint32_t* d_base;
        CK(hipMalloc(&d_base, nr * 4ull));
        CK(hipMemcpy(d_base, base.data(), nr * 4ull, hipMemcpyHostToDevice));
        char name[64];
        snprintf(name, sizeof name, "64B entries in random runs of %u", run);
        const uint32_t nn = nr * run;
        timeit(name, [&] { hipLaunchKernelGGL(k_runs, dim3((nn + 255) / 256), dim3(256), 0, 0, (const uint4*)buf, d_base, run, nn, d_out); }, 64);
        CK(hipFree(d_base));
    }
    return 0;
}
