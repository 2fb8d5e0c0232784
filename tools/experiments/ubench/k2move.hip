// Write side of the C4 lever (read side: k2local.hip) -- diagnostic, not the product.
// What it costs to move 10.5M 32-B update units from record order into super-partition runs (S
// supers of P / S partitions each, units in record order inside a run per chunk): one chunk of CH
// units per workgroup, coalesced loads, an LDS counting sort by super (ranks by LDS atomics: the
// order inside a run is not kept stable here, which only makes this cheaper than the real move), and
// each super's run written contiguously at its offset (super-major, chunk-minor, precomputed on the
// host as K1's histograms would give it).  Baseline: the same units copied in order.
// Build: hipcc -O3 --offload-arch=gfx950 -o k2move k2move.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static unsigned long long sm(unsigned long long& s) {
    unsigned long long z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(512) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t n16) {
    for (uint32_t i = blockIdx.x * 512u + threadIdx.x; i < n16; i += gridDim.x * 512u) out[i] = in[i];
}

template <uint32_t CH, uint32_t S>
__global__ __launch_bounds__(512) void k_move(const uint4* __restrict__ units, const uint16_t* __restrict__ sup,
                                              const uint32_t* __restrict__ off, uint4* __restrict__ out, uint32_t N) {
    __shared__ uint4 st[2 * CH];
    __shared__ uint16_t sp[CH];
    __shared__ uint32_t hist[S], base[S];
    constexpr uint32_t K = CH / 512u;
    const uint32_t c = blockIdx.x, u0 = c * CH, cnt = min(CH, N - u0), tid = threadIdx.x;
    for (uint32_t s = tid; s < S; s += 512u) hist[s] = 0u;
    __syncthreads();
    uint32_t rank[K], sv[K];
    uint4 a[K], b[K];
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t i = tid + k * 512u;
        if (i < cnt) {
            sv[k] = sup[u0 + i];
            a[k] = units[2ull * (u0 + i)];
            b[k] = units[2ull * (u0 + i) + 1];
            rank[k] = atomicAdd(&hist[sv[k]], 1u);
        }
    }
    __syncthreads();
    if (tid < 64u) {  // exclusive scan of the S counts by one wave
        uint32_t carry = 0u;
        for (uint32_t s0 = 0; s0 < S; s0 += 64u) {
            const uint32_t v = s0 + tid < S ? hist[s0 + tid] : 0u;
            uint32_t x = v;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (tid >= (uint32_t)o) x += y;
            }
            if (s0 + tid < S) base[s0 + tid] = carry + x - v;
            carry += __shfl(x, 63, 64);
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t i = tid + k * 512u;
        if (i < cnt) {
            const uint32_t pos = base[sv[k]] + rank[k];
            st[2 * pos] = a[k];
            st[2 * pos + 1] = b[k];
            sp[pos] = (uint16_t)sv[k];
        }
    }
    __syncthreads();
    for (uint32_t pos = tid; pos < cnt; pos += 512u) {
        const uint32_t s = sp[pos];
        const uint32_t dst = off[(size_t)c * S + s] + (pos - base[s]);
        out[2ull * dst] = st[2 * pos];
        out[2ull * dst + 1] = st[2 * pos + 1];
    }
}

template <uint32_t CH, uint32_t S>
static void run(const uint4* d_units, uint4* d_out, const std::vector<uint32_t>& part, uint32_t N, uint32_t P) {
    const uint32_t chunks = (N + CH - 1) / CH;
    std::vector<uint16_t> sup(N);
    for (uint32_t u = 0; u < N; ++u) sup[u] = (uint16_t)(part[u] / (P / S));
    std::vector<uint32_t> cnt((size_t)chunks * S, 0), off((size_t)chunks * S);
    for (uint32_t u = 0; u < N; ++u) cnt[(size_t)(u / CH) * S + sup[u]]++;
    uint32_t acc = 0;
    for (uint32_t s = 0; s < S; ++s)
        for (uint32_t c = 0; c < chunks; ++c) {
            off[(size_t)c * S + s] = acc;
            acc += cnt[(size_t)c * S + s];
        }
    uint16_t* d_sup;
    uint32_t* d_off;
    CK(hipMalloc(&d_sup, (size_t)N * 2));
    CK(hipMalloc(&d_off, off.size() * 4));
    CK(hipMemcpy(d_sup, sup.data(), (size_t)N * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9f, sum = 0.f;
    const int reps = 20;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_move<CH, S>), dim3(chunks), dim3(512), 0, 0, d_units, d_sup, d_off, d_out, N);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) { best = std::min(best, ms); sum += ms; }
    }
    // check: every unit landed (units hold their index in word 0)
    std::vector<uint4> h((size_t)N * 2);
    CK(hipMemcpy(h.data(), d_out, (size_t)N * 32, hipMemcpyDeviceToHost));
    std::vector<char> seen(N, 0);
    std::vector<uint32_t> sbeg(S);  // super s starts at its chunk-0 offset
    for (uint32_t s = 0; s < S; ++s) sbeg[s] = off[s];
    uint32_t bad = 0;
    for (uint32_t i = 0; i < N; ++i) {
        const uint32_t u = h[2ull * i].x;
        const uint32_t s = (uint32_t)(std::upper_bound(sbeg.begin(), sbeg.end(), i) - sbeg.begin()) - 1u;
        if (u >= N || seen[u] || sup[u] != s) ++bad;
        else seen[u] = 1;
    }
    printf("move   CH=%-5u S=%-4u  best %.1f us  mean %.1f us  (%u misplaced)\n", CH, S, best * 1e3f, sum / reps * 1e3f, bad);
    CK(hipFree(d_sup));
    CK(hipFree(d_off));
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 10485760u, P = 4096u;
    unsigned long long seed = 12345;
    std::vector<uint32_t> part(N);
    for (uint32_t u = 0; u < N; ++u) part[u] = (uint32_t)(sm(seed) % P);
    std::vector<uint4> hu((size_t)N * 2);
    for (uint32_t u = 0; u < N; ++u) {
        hu[2ull * u] = make_uint4(u, part[u], 1u, 2u);
        hu[2ull * u + 1] = make_uint4(3u, 4u, 5u, 6u);
    }
    uint4 *d_units, *d_out;
    CK(hipMalloc(&d_units, (size_t)N * 32));
    CK(hipMalloc(&d_out, (size_t)N * 32));
    CK(hipMemcpy(d_units, hu.data(), (size_t)N * 32, hipMemcpyHostToDevice));
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9f;
        for (int r = 0; r < 22; ++r) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_copy, dim3(2048), dim3(512), 0, 0, d_units, d_out, N * 2u);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) best = std::min(best, ms);
        }
        printf("copy   in order          best %.1f us  (%u units, 2 x %.0f MB)\n", best * 1e3f, N, N * 32.0 / 1e6);
    }
    run<2048, 128>(d_units, d_out, part, N, P);
    run<4096, 128>(d_units, d_out, part, N, P);
    run<4096, 256>(d_units, d_out, part, N, P);
    run<2048, 64>(d_units, d_out, part, N, P);
    return 0;
}
