// fb_compact.hip -- batch-wide (dense) output: the scan of the segment counts and the copy of a
// segmented batch into dense arrays.
//
// fb_parse_classify_dev / fb_process_parsed_dev / fb_process_dev promise the reference's
// emission order with no gaps: class-SESSION records packed in packet order, DNS side records
// likewise (what a caller iterating frames one by one through parse_packet_pcap +
// process_parsed_packet, src/capture.rs:1036-1061, would see).  Frame batches take the
// single-pass k_parse_dense (fb_parse.hip); parsed-packet batches run k_parse_seg twice
// (fb_capi.hip parse_dense): pass 1 counts each 64-frame segment (and writes classes + stats),
// k_seg_scan (one pass, decoupled look-back) turns the counts into batch-wide offsets, pass 2
// re-parses (the frames of a 1M-frame batch are still in the Infinity Cache) and stores every
// record at its final position.  fb_seg_compact_dev instead copies an existing segmented batch
// (k_seg_compact: one wavefront per segment, its records from the segment head, its DNS records
// from the tail).  No kernel here or in the parse waits on another workgroup, so the dense path
// is as safe on a shared GPU as the segmented one.
//   scan: 4 B per segment read, 8 B per segment written (+ 8 B of status per 1024-segment tile).
//   copy: 56 B per SESSION record and 16 B per DNS record read and written.
#include "fb_internal.h"

namespace fbk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kCompactWaves = 4;
constexpr uint32_t kSegOutBytes = 64u * 56u;  // one segment of k_parse_seg output
constexpr uint32_t kOob = 0x80000000u;        // buffer offset past every resource: store dropped

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanPer = 4;                          // segment words per thread
constexpr uint32_t kScanTile = kScanThreads * kScanPer;   // segments per scan workgroup

// count word -> (n_session, n_dns) packed as n_session | n_dns << 32 (sums stay exact: < 2^27 each)
__device__ __forceinline__ unsigned long long seg_pair(uint32_t w) {
    return (unsigned long long)(w & 0xFFFFu) | ((unsigned long long)(w >> 16) << 32);
}
// tile status word [epoch:8 | P:1 | A:1 | n_dns:27 | n_session:27]: A = the tile's own sum is
// published, P = its inclusive prefix is
constexpr unsigned long long kStA = 1ull << 54, kStP = 1ull << 55, kSt27 = (1ull << 27) - 1ull;
__device__ __forceinline__ unsigned long long st_word(uint32_t ep, unsigned long long flag, unsigned long long pair) {
    return ((unsigned long long)ep << 56) | flag | (pair & kSt27) | (((pair >> 32) & kSt27) << 27);
}
__device__ __forceinline__ unsigned long long st_pair(unsigned long long w) {
    return (w & kSt27) | (((w >> 27) & kSt27) << 32);
}

// Single-pass exclusive scan of the segment count words into pre[] (u64 n_session | n_dns << 32):
// decoupled look-back over tiles of kScanTile segments whose order is a ticket taken at block
// start, so a tile only ever waits for tiles that running blocks already own -- no residency
// assumption.  Status words are epoch-tagged (no per-call zeroing); the block that takes the last
// ticket resets the ticket counter for the next call.
__global__ __launch_bounds__(kScanThreads) void k_seg_scan(const uint32_t* seg, uint32_t nseg, unsigned long long* pre,
                                                           unsigned long long* status, uint32_t* ticket, uint32_t ep,
                                                           uint32_t nblk, uint32_t* err) {
    __shared__ uint32_t s_t;
    __shared__ unsigned long long s_w[kScanThreads / 64];
    __shared__ unsigned long long s_excl;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    if (tid == 0u) {
        const uint32_t t = atomicAdd(ticket, 1u);
        if (t == nblk - 1u) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_t = t;
    }
    __syncthreads();
    const uint32_t t = s_t;
    const uint32_t first = t * kScanTile + tid * kScanPer;
    uint32_t w[kScanPer];
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) w[j] = first + j < nseg ? seg[first + j] : 0u;
    unsigned long long mine = 0ull;
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) mine += seg_pair(w[j]);
    unsigned long long inc = mine;  // inclusive over the wave, then the block
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) s_w[wave] = inc;
    __syncthreads();
    unsigned long long before_wave = 0ull, agg = 0ull;
#pragma unroll
    for (uint32_t k = 0; k < kScanThreads / 64u; ++k) {
        before_wave += k < wave ? s_w[k] : 0ull;
        agg += s_w[k];
    }
    if (wave == 0u) {
        unsigned long long excl = 0ull;
        if (t == 0u) {
            if (lane == 0u) __hip_atomic_store(status, st_word(ep, kStP, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0u) __hip_atomic_store(status + t, st_word(ep, kStA, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)t;  // window: tiles j-1-lane
            uint32_t spins = 0u;
            for (;;) {
                const int64_t idx = j - 1 - (int64_t)lane;
                auto probe = [&]() {
                    return idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : st_word(ep, kStP, 0ull);
                };
                unsigned long long v = probe();
                while (__ballot((uint32_t)(v >> 56) != ep || !(v & (kStA | kStP))) != 0ull) {
                    if (++spins > (1u << 22)) {  // never expected: a lower ticket's block stalled
                        if (lane == 0u) atomicOr(err, 2u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    if ((uint32_t)(v >> 56) != ep || !(v & (kStA | kStP))) v = probe();
                }
                const unsigned long long pm = __ballot((v & kStP) != 0ull);
                const uint32_t stop = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;  // nearest inclusive
                unsigned long long part = lane <= stop ? st_pair(v) : 0ull;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
                excl += part;
                if (pm || spins > (1u << 22)) break;
                j -= 64;
            }
            if (lane == 0u)
                __hip_atomic_store(status + t, st_word(ep, kStP, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0u) s_excl = excl;
    }
    __syncthreads();
    unsigned long long run = s_excl + before_wave + inc - mine;
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

hipError_t launch_seg_scan(const uint32_t* seg, uint32_t nseg, unsigned long long* pre, const SegScanScratch& sc,
                           hipStream_t s) {
    if (nseg == 0u) return hipSuccess;
    const uint32_t nblk = seg_scan_tiles(nseg);
    hipLaunchKernelGGL(k_seg_scan, dim3(nblk), dim3(kScanThreads), 0, s, seg, nseg, pre, sc.status, sc.ticket, sc.epoch,
                       nblk, sc.err);
    return hipGetLastError();
}

uint32_t seg_scan_tiles(uint32_t nseg) { return (nseg + kScanTile - 1) / kScanTile; }

hipError_t launch_seg_compact(const fb_pkt_out* seg_out, const uint32_t* seg, uint32_t nseg, unsigned long long* pre,
                              const SegScanScratch& sc, fb_pkt_out* out, fb_dns_out* dns, hipStream_t s) {
    if (nseg == 0u || (!out && !dns)) return hipSuccess;
    hipError_t e = launch_seg_scan(seg, nseg, pre, sc, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_compact, dim3((nseg + kCompactWaves - 1) / kCompactWaves), dim3(64 * kCompactWaves), 0, s,
                       reinterpret_cast<const uint8_t*>(seg_out), seg, (const unsigned long long*)pre, nseg, out, dns);
    return hipGetLastError();
}

}  // namespace fbk
