// fb_compact.hip -- batch-wide (dense) output: the scan of the segment counts and the copy of a
// segmented batch into dense arrays.
//
// fb_parse_classify_dev / fb_process_parsed_dev / fb_process_dev promise the reference's
// emission order with no gaps: class-SESSION records packed in packet order, DNS side records
// likewise (what a caller iterating frames one by one through parse_packet_pcap +
// process_parsed_packet, src/capture.rs:1036-1061, would see).  They run k_parse_seg twice
// (fb_capi.hip parse_dense): pass 1 counts each 64-frame segment (and writes classes + stats),
// k_seg_tile_sums / k_seg_scan turn the counts into per-segment batch-wide offsets, pass 2
// re-parses (the frames of a 1M-frame batch are still in the Infinity Cache) and stores every
// record at its final position.  fb_seg_compact_dev instead copies an existing segmented batch
// (k_seg_compact: one wavefront per segment, its records from the segment head, its DNS records
// from the tail).  No kernel here or in the parse waits on another workgroup, so the dense path
// is as safe on a shared GPU as the segmented one.
//   scan: 4 B per segment read twice, 8 B per segment written (+ 8 B per 4096-segment tile).
//   copy: 56 B per SESSION record and 16 B per DNS record read and written.
#include "fb_internal.h"

namespace fbk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kCompactWaves = 4;
constexpr uint32_t kSegOutBytes = 64u * 56u;  // one segment of k_parse_seg output
constexpr uint32_t kOob = 0x80000000u;        // buffer offset past every resource: store dropped

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanPer = 16;                         // segment words per thread
constexpr uint32_t kScanTile = kScanThreads * kScanPer;   // segments per scan workgroup

// count word -> (n_session, n_dns) packed as n_session | n_dns << 32 (sums stay exact: < 2^27 each)
__device__ __forceinline__ unsigned long long seg_pair(uint32_t w) {
    return (unsigned long long)(w & 0xFFFFu) | ((unsigned long long)(w >> 16) << 32);
}

__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63u) == 0u) red[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long t = 0ull;
#pragma unroll
    for (uint32_t w = 0; w < kScanThreads / 64u; ++w) t += red[w];
    __syncthreads();
    return t;
}

// Per tile of kScanTile segments: the sum of its count pairs.
__global__ __launch_bounds__(kScanThreads) void k_seg_tile_sums(const uint32_t* seg, uint32_t nseg,
                                                                unsigned long long* tsum) {
    __shared__ unsigned long long red[kScanThreads / 64];
    const uint32_t base = blockIdx.x * kScanTile;
    unsigned long long v = 0ull;
    for (uint32_t j = threadIdx.x; j < kScanTile; j += kScanThreads)
        if (base + j < nseg) v += seg_pair(seg[base + j]);
    v = block_sum(v, red);
    if (threadIdx.x == 0u) tsum[blockIdx.x] = v;
}

// Exclusive prefix of every segment: the tiles before this one (summed here from tsum) + the
// block scan of this tile (each thread owns kScanPer consecutive segments).
__global__ __launch_bounds__(kScanThreads) void k_seg_scan(const uint32_t* seg, uint32_t nseg,
                                                           const unsigned long long* tsum, unsigned long long* pre) {
    __shared__ unsigned long long red[kScanThreads / 64];
    __shared__ unsigned long long wpre[kScanThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    unsigned long long before = 0ull;
    for (uint32_t t = tid; t < blockIdx.x; t += kScanThreads) before += tsum[t];
    before = block_sum(before, red);
    const uint32_t first = blockIdx.x * kScanTile + tid * kScanPer;
    uint32_t w[kScanPer];
    unsigned long long mine = 0ull;
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
        w[j] = first + j < nseg ? seg[first + j] : 0u;
        mine += seg_pair(w[j]);
    }
    // inclusive scan of `mine` over the wave, then over the waves
    unsigned long long inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) wpre[wave] = inc;
    __syncthreads();
    unsigned long long run = before + inc - mine;
    for (uint32_t k = 0; k < wave; ++k) run += wpre[k];
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
        if (first + j < nseg) pre[first + j] = run;
        run += seg_pair(w[j]);
    }
}

__global__ __launch_bounds__(64 * kCompactWaves) void k_seg_compact(const uint8_t* seg_out, const uint32_t* seg,
                                                                    const unsigned long long* pre, uint32_t nseg,
                                                                    fb_pkt_out* out, fb_dns_out* dns) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t sg = blockIdx.x * kCompactWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (sg >= nseg) return;  // wave-uniform
    const uint32_t cnt = seg[sg], cs = cnt & 0xFFFFu, cd = cnt >> 16;
    const unsigned long long p = pre[sg];
    const uint32_t bs = (uint32_t)p, bd = (uint32_t)(p >> 32);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(seg_out + (size_t)sg * kSegOutBytes), (short)0, (int)kSegOutBytes, 0x00020000);
    if (out && cs) {
        // record bytes [0, 56 cs) of the segment -> bytes [56 bs, ..) of out.  56 bs is 16-B
        // aligned when bs is even; otherwise the first 8-B word goes alone and the 16-B body
        // stores stay aligned (the matching loads are 8-B aligned, which buffer loads allow).
        const uint32_t words = cs * 7u, head = bs & 1u, body = (words - head) >> 1;
        uint8_t* dst = reinterpret_cast<uint8_t*>(out) + (size_t)bs * 56u;
        const __amdgpu_buffer_rsrc_t rdst = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)(words * 8u), 0x00020000);
        for (uint32_t c = lane; c < body; c += 64u) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, head * 8u + c * 16u, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, rdst, head * 8u + c * 16u, 0, 0);
        }
        const bool single_head = head && lane == 0u;
        const bool single_tail = ((words - head) & 1u) && lane == 1u;
        if (single_head || single_tail) {
            const uint32_t w = single_head ? 0u : words - 1u;
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, w * 8u, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(v, rdst, w * 8u, 0, 0);
        }
    }
    if (dns && cd) {
        for (uint32_t j = lane; j < cd; j += 64u) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, kSegOutBytes - 16u * (j + 1u), 0, 0);
            *reinterpret_cast<u32x4*>(dns + bd + j) = v;
        }
    }
}

hipError_t launch_seg_scan(const uint32_t* seg, uint32_t nseg, unsigned long long* pre, unsigned long long* tsum,
                           hipStream_t s) {
    if (nseg == 0u) return hipSuccess;
    const uint32_t tiles = (nseg + kScanTile - 1) / kScanTile;
    if (tiles > 1u) hipLaunchKernelGGL(k_seg_tile_sums, dim3(tiles), dim3(kScanThreads), 0, s, seg, nseg, tsum);
    hipLaunchKernelGGL(k_seg_scan, dim3(tiles), dim3(kScanThreads), 0, s, seg, nseg, (const unsigned long long*)tsum, pre);
    return hipGetLastError();
}

uint32_t seg_scan_tiles(uint32_t nseg) { return (nseg + kScanTile - 1) / kScanTile; }

hipError_t launch_seg_compact(const fb_pkt_out* seg_out, const uint32_t* seg, uint32_t nseg, unsigned long long* pre,
                              unsigned long long* tsum, fb_pkt_out* out, fb_dns_out* dns, hipStream_t s) {
    if (nseg == 0u || (!out && !dns)) return hipSuccess;
    hipError_t e = launch_seg_scan(seg, nseg, pre, tsum, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_compact, dim3((nseg + kCompactWaves - 1) / kCompactWaves), dim3(64 * kCompactWaves), 0, s,
                       reinterpret_cast<const uint8_t*>(seg_out), seg, (const unsigned long long*)pre, nseg, out, dns);
    return hipGetLastError();
}

}  // namespace fbk
