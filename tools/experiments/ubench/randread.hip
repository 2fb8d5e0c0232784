// Random 32-B read rate vs footprint (diagnostic, not the product): N reads of 2 x uint4 at
// pseudo-random 32-B-aligned offsets inside a buffer of `span` bytes, one read per lane per
// iteration, K independent reads in flight per lane.  Prints GB/s (of 32-B units) and Greads/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

template <int K>
__global__ __launch_bounds__(256) void k_rand(const uint4* buf, unsigned long long units, unsigned long long n,
                                              unsigned long long cluster, uint4* out) {
    const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x, nt = gridDim.x * 256ull;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (unsigned long long i0 = tid; i0 < n; i0 += nt * K) {
        uint4 a[K], b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned long long i = i0 + k * nt;
            // cluster > 1: consecutive reads (i / cluster) share a random 'row' of cluster units
            const unsigned long long base = (mix(i / cluster) % (units / cluster)) * cluster;
            const unsigned long long u = base + (i % cluster);
            a[k] = buf[2 * u];
            b[k] = buf[2 * u + 1];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc.x ^= a[k].x ^ b[k].y;
            acc.y += a[k].y ^ b[k].x;
        }
    }
    if (acc.x == 0x12345678u) out[tid & ((1u << 20) - 1u)] = acc;
}


// Two lanes per unit: lanes 2i and 2i+1 read the two 16-B halves of unit(2i) in one instruction and
// of unit(2i+1) in the next (one line request per unit instead of two), then swap halves.
__global__ __launch_bounds__(256) void k_rand_pair(const uint4* buf, unsigned long long units, unsigned long long n,
                                                   uint4* out) {
    const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x, nt = gridDim.x * 256ull;
    const uint32_t lane = threadIdx.x & 63u, odd = lane & 1u;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (unsigned long long i0 = tid; i0 < n; i0 += nt * 4) {
        uint4 a[4], b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned long long i = i0 + k * nt;
            const unsigned long long u = mix(i) % units;                  // this lane's unit
            const unsigned long long up = __shfl_xor((long long)u, 1, 64);  // the partner's
            const unsigned long long ue = odd ? up : u, uo = odd ? u : up;  // unit of lane 2i, of 2i+1
            a[k] = buf[2 * ue + odd];  // instruction 1: unit(2i), half = lane parity
            b[k] = buf[2 * uo + odd];  // instruction 2: unit(2i+1)
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // lane 2i keeps a (half 0 of its unit) and takes the partner's a (half 1);
            // lane 2i+1 keeps b (half 1 of its unit) and takes the partner's b (half 0)
            const uint4 mine = odd ? b[k] : a[k];
            const uint4 give = odd ? a[k] : b[k];
            uint4 other;
            other.x = __shfl_xor((int)give.x, 1, 64);
            other.y = __shfl_xor((int)give.y, 1, 64);
            other.z = __shfl_xor((int)give.z, 1, 64);
            other.w = __shfl_xor((int)give.w, 1, 64);
            acc.x ^= mine.x ^ other.y;
            acc.y += mine.y ^ other.x;
        }
    }
    if (acc.x == 0x12345678u) out[tid & ((1u << 20) - 1u)] = acc;
}

int main() {
    const unsigned long long spans[] = {32ull << 20, 128ull << 20, 336ull << 20, 672ull << 20, 2048ull << 20};
    const unsigned long long n = 10ull << 20;
    uint4* buf;
    uint4* out;
    hipMalloc(&buf, 2048ull << 20);
    hipMalloc(&out, 1 << 24);
    hipMemset(buf, 1, 2048ull << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (unsigned long long cl : {1ull, 4ull, 64ull}) {
        for (unsigned long long span : spans) {
            const unsigned long long units = span / 32;
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_rand<4>, dim3(8192), dim3(256), 0, 0, buf, units, n, cl, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("cluster %3llu span %5llu MB: %8.1f us  %6.2f Greads/s  %7.1f GB/s\n", cl, span >> 20, best * 1e3,
                   n / (best * 1e-3) / 1e9, n * 32.0 / (best * 1e-3) / 1e9);
        }
    }
    for (unsigned long long span : spans) {
        const unsigned long long units = span / 32;
        float best = 1e9f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_rand_pair, dim3(8192), dim3(256), 0, 0, buf, units, n, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("paired      span %5llu MB: %8.1f us  %6.2f Greads/s  %7.1f GB/s\n", span >> 20, best * 1e3,
               n / (best * 1e-3) / 1e9, n * 32.0 / (best * 1e-3) / 1e9);
    }
    return 0;
}
