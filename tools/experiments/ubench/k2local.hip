// K2 unit-read locality microbenchmark (diagnostic, not the product).  DESIGN §9.1's C4 lever:
// K2 (k_flow_apply) reads one 32-B update unit per record, each from a line of its own, and is paced
// by the fabric's ~33-45 G line requests/s.  This measures the same gather with the units laid out
// per "super-partition" (a group of partitions) and the partitions of a super dealt to workgroups of
// ONE XCD (blocks b and b + 8 share an XCD under round-robin dispatch), so a line's four units are
// fetched into that XCD's L2 once and the other partitions' workgroups hit it there.
//
// Layouts (10.5M units, P = 4096 partitions of a 2^21-slot table, units' partitions uniform random):
//   packed   units in record order (the product's per-segment packing), partition random per unit
//   super    units grouped by super = partition / (P / S), random order inside a super
// Mappings (workgroup i -> partition):  ident  p = i;  xcd  i % 8 = the super's XCD, supers of an
// XCD in order.  Each workgroup reads its partition's index words (contiguous) and gathers the
// units (two 16-B loads), two units per thread in flight, like K2's pipeline.
// Build: hipcc -O3 --offload-arch=gfx950 -o k2local k2local.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <numeric>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static unsigned long long sm(unsigned long long& s) {
    unsigned long long z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int U>
__global__ __launch_bounds__(512) void k_gather(const uint4* __restrict__ units, const uint32_t* __restrict__ idx,
                                                const uint32_t* __restrict__ pstart, uint32_t P, uint32_t S,
                                                uint32_t xcd_map, uint4* out) {
    extern __shared__ uint32_t pad[];  // launched with K2's 72 KB to get its two workgroups per CU
    if (threadIdx.x == 1023u) pad[0] = 0u;
    const uint32_t i = blockIdx.x;
    uint32_t p = i;
    if (xcd_map == 2u) {  // XCD-contiguous: XCD x (blocks i % 8 == x) takes partitions [x P/8, (x+1) P/8) in order
        p = (i % 8u) * (P / 8u) + i / 8u;
    } else if (xcd_map) {
        const uint32_t per = P / S, x = i % 8u, k = i / 8u;  // XCD x: supers x, x + 8, ..., in order
        const uint32_t s = x + 8u * (k / per);
        p = s * per + k % per;
    }
    const uint32_t a = pstart[p], b = pstart[p + 1];
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t e = a + threadIdx.x; e < b; e += U * 512u) {
        uint32_t u[U];
#pragma unroll
        for (int k = 0; k < U; ++k) u[k] = e + k * 512u < b ? idx[e + k * 512u] : idx[e];
        uint4 x[U], y[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            x[k] = units[2ull * u[k]];
            y[k] = units[2ull * u[k] + 1];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            acc.x ^= x[k].x + y[k].y;
            acc.y += x[k].w ^ y[k].x;
            acc.z ^= y[k].z + x[k].y;
            acc.w += y[k].w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[blockIdx.x * 512u + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 10485760u, P = 4096u;
    const int reps = 20;
    unsigned long long seed = 12345;
    std::vector<uint32_t> part(N);
    for (uint32_t u = 0; u < N; ++u) part[u] = (uint32_t)(sm(seed) % P);
    uint4* d_units;
    CK(hipMalloc(&d_units, (size_t)N * 32));
    CK(hipMemset(d_units, 1, (size_t)N * 32));
    uint4* d_out;
    CK(hipMalloc(&d_out, (size_t)P * 512 * 16));
    uint32_t *d_idx, *d_ps;
    CK(hipMalloc(&d_idx, (size_t)N * 4));
    CK(hipMalloc(&d_ps, (size_t)(P + 1) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipFuncSetAttribute((const void*)k_gather<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024));
    CK(hipFuncSetAttribute((const void*)k_gather<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024));
    const uint32_t Ss[] = {0u, 64u, 128u, 256u, 4096u};  // 0: packed layout; P: contiguous per partition
    for (uint32_t S : Ss) {
        // the layout: position of each record's unit
        std::vector<uint32_t> pos(N);
        if (S == 0) {
            std::iota(pos.begin(), pos.end(), 0u);
        } else {
            const uint32_t per = P / S;
            std::vector<uint32_t> cnt(S + 1, 0);
            for (uint32_t u = 0; u < N; ++u) cnt[part[u] / per + 1]++;
            for (uint32_t s = 0; s < S; ++s) cnt[s + 1] += cnt[s];
            for (uint32_t u = 0; u < N; ++u) pos[u] = cnt[part[u] / per]++;  // record order inside a super
        }
        // per-partition lists (CSR), records in order
        std::vector<uint32_t> ps(P + 1, 0), idx(N);
        for (uint32_t u = 0; u < N; ++u) ps[part[u] + 1]++;
        for (uint32_t p = 0; p < P; ++p) ps[p + 1] += ps[p];
        std::vector<uint32_t> cur(ps.begin(), ps.end() - 1);
        for (uint32_t u = 0; u < N; ++u) idx[cur[part[u]]++] = pos[u];
        CK(hipMemcpy(d_idx, idx.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_ps, ps.data(), (size_t)(P + 1) * 4, hipMemcpyHostToDevice));
        for (uint32_t v = 0; v < (S ? 2u : 5u); ++v) {
          const uint32_t xm = S ? v : 0u;
          // packed layout variants: units in flight per thread (2 / 4) x free occupancy / K2's 72 KB LDS
          const int U = (S || v == 0 || v == 1 || v == 3) ? 2 : 4;
          const size_t lds = (!S && v >= 3) ? 72u * 1024u : 0u;
          if (!S && v == 1) continue;
          {
            float best = 1e9f, sum = 0.f;
            for (int r = 0; r < reps + 2; ++r) {
                CK(hipEventRecord(e0));
                if (U == 2)
                    hipLaunchKernelGGL(k_gather<2>, dim3(P), dim3(512), lds, 0, d_units, d_idx, d_ps, P, S ? S : 1u, xm, d_out);
                else
                    hipLaunchKernelGGL(k_gather<4>, dim3(P), dim3(512), lds, 0, d_units, d_idx, d_ps, P, S ? S : 1u, xm, d_out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) { best = std::min(best, ms); sum += ms; }
            }
            printf("%-7s S=%-4u map=%-5s inflight=%d lds=%zuK  units %u  best %.1f us  mean %.1f us  %.1f G units/s\n",
                   S ? "super" : "packed", S, xm ? "xcd" : "ident", U, lds >> 10, N, best * 1e3f, sum / reps * 1e3f,
                   N / (best * 1e-3f) / 1e9f);
          }
        }
    }
    // layouts of the fused parse: units sorted by partition inside groups of G consecutive records
    // (G = 64: the product's per-segment sort; 256 / 1024: a wave's 4 / a block's 16 segments)
    // (BK > 1: sorted by partition / BK only -- the bucket of 64 consecutive partitions one XCD's K2
    // workgroups hold at once under the XCD-contiguous mapping -- order inside a bucket arbitrary)
    for (uint32_t GB : {64u, 256u, 1024u, 256u | (64u << 16), 320u | (64u << 16), 384u | (64u << 16)}) {
        const uint32_t G = GB & 0xFFFFu, BK = GB >> 16 ? GB >> 16 : 1u;
        std::vector<uint32_t> pos(N), ord(G);
        for (uint32_t g0 = 0; g0 < N; g0 += G) {
            const uint32_t m = std::min(G, N - g0);
            for (uint32_t k = 0; k < m; ++k) ord[k] = g0 + k;
            std::stable_sort(ord.begin(), ord.begin() + m, [&](uint32_t x, uint32_t y) {
                return part[x] / BK < part[y] / BK || (part[x] / BK == part[y] / BK && BK > 1u && (x * 2654435761u) < (y * 2654435761u));
            });
            for (uint32_t k = 0; k < m; ++k) pos[ord[k]] = g0 + k;
        }
        std::vector<uint32_t> ps(P + 1, 0), idx(N);
        for (uint32_t u = 0; u < N; ++u) ps[part[u] + 1]++;
        for (uint32_t q = 0; q < P; ++q) ps[q + 1] += ps[q];
        std::vector<uint32_t> cur(ps.begin(), ps.end() - 1);
        for (uint32_t u = 0; u < N; ++u) idx[cur[part[u]]++] = pos[u];
        CK(hipMemcpy(d_idx, idx.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_ps, ps.data(), (size_t)(P + 1) * 4, hipMemcpyHostToDevice));
        for (uint32_t xm : {0u, 2u}) {
            float best = 1e9f, sum = 0.f;
            for (int r = 0; r < reps + 2; ++r) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_gather<2>, dim3(P), dim3(512), 72u * 1024u, 0, d_units, d_idx, d_ps, P, 1u, xm, d_out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) { best = std::min(best, ms); sum += ms; }
            }
            printf("sorted G=%-5u key=part/%-3u map=%-6s lds=72K  units %u  best %.1f us  mean %.1f us  %.1f G units/s\n", G,
                   BK, xm ? "xcdrun" : "ident", N, best * 1e3f, sum / reps * 1e3f, N / (best * 1e-3f) / 1e9f);
        }
    }
    return 0;
}
