// fb_hist.hip -- per-flow history characters of one flow-table update, in packet order.
//
// The reference appends map_tcp_flags(..) to the flow's `history` String for every TCP packet
// (src/packets.rs:187-198 occupied, 410-426 vacant), so a flow's history is its TCP packets'
// characters in arrival order.  k_flow_apply (fb_flow.hip) records the table slot of every
// record slot of the batch via `rec_flow` (entry position) and `ent_slot` / `agg_slot`; here the batch's TCP records are stably sorted by that
// slot, which groups each flow's characters into one run while keeping packet order inside it:
//   k_hist_keys : key[i] = rec_flow[i] for a valid record with FB_META_HAS_FLAGS, else the
//                 sentinel (= table capacity, sorts last); value[i] = the record's hist_char;
//                 counts the keyed records into *n_hist.
//   radix sort  : rocPRIM's stable LSD radix sort over log2(capacity)+1 key bits, pairs
//                 (u32 slot, u8 char) -> the caller's d_hist_slot / d_hist.
// Bytes per record: 4 (the fused parse's per-record word -- partition, history character,
// has_flags -- or, without it, the record's word 12, which at 56-B stride costs its sector) + 4
// (rec_flow) read, 5 written, then the sort's passes.  C4: 160 -> 92 us with the fused word.
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "fb_internal.h"

namespace fbk {

__global__ __launch_bounds__(256) void k_hist_keys(const HistParams P) {
    __shared__ uint32_t wcnt[4];
    const uint32_t n = P.seg ? P.n_slots : (uint32_t)min(P.stats->n_session, (unsigned long long)P.n_slots);
    uint32_t cnt = 0u;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < P.n_slots; i += stride) {
        bool keyed = false;
        uint32_t ch = 0u;
        if (i < n && (!P.seg || (i & 63u) < (P.seg[i >> 6] & 0xFFFFu))) {
            if (P.rec_part) {  // the fused parse's word: 4 B per slot instead of the 56-B record's word 12
                const uint32_t w = P.rec_part[i];
                keyed = (w >> 24) & 1u;
                ch = (w >> 16) & 0xFFu;
            } else {
                const uint32_t w = reinterpret_cast<const uint32_t*>(P.recs + i)[12];  // flags|meta|hist_char
                keyed = ((w >> 8) & FB_META_HAS_FLAGS) != 0u;
                ch = (w >> 16) & 0xFFu;
            }
        }
        uint32_t slot = P.sentinel;
        if (keyed) {
            const uint32_t v = P.rec_flow[i];  // entry position, or a k_flow_combine id
            slot = (v & kRecFlowCombined) ? P.agg_slot[v & ~kRecFlowCombined] : P.ent_slot[v];
        }
        P.keys[i] = slot;
        P.vals[i] = (uint8_t)ch;
        cnt += keyed;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63u) == 0u) wcnt[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (t) atomicAdd(P.n_hist, t);
    }
}

#ifndef FB_HIST_RADIX_BITS
#define FB_HIST_RADIX_BITS 0  // 0: rocPRIM's gfx950 default (8 bits per onesweep pass)
#endif
#ifndef FB_HIST_SORT_BLOCK
#define FB_HIST_SORT_BLOCK 1024
#endif
#ifndef FB_HIST_SORT_IPT
#define FB_HIST_SORT_IPT 8
#endif
#if FB_HIST_RADIX_BITS
using HistSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                        rocprim::kernel_config<FB_HIST_SORT_BLOCK, FB_HIST_SORT_IPT>,
                                        FB_HIST_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;
#else
using HistSortConfig = rocprim::default_config;
#endif

static uint32_t key_bits(uint32_t sentinel) {
    uint32_t b = 1u;
    while (b < 32u && (1ull << b) <= sentinel) ++b;
    return b;
}

hipError_t flow_history_temp_bytes(uint32_t n_slots, uint32_t sentinel, size_t* bytes) {
    return rocprim::radix_sort_pairs<HistSortConfig>(nullptr, *bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const uint8_t*)nullptr, (uint8_t*)nullptr, (size_t)n_slots, 0u,
                                     key_bits(sentinel));
}

hipError_t launch_flow_history(const HistParams& p, void* temp, size_t temp_bytes, uint32_t* hist_slot,
                               uint8_t* hist, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.n_hist, 0, 4, s);
    if (e != hipSuccess || p.n_slots == 0u) return e;
    const uint32_t grid = std::min<uint32_t>((p.n_slots + 255u) / 256u, 2048u);
    hipLaunchKernelGGL(k_hist_keys, dim3(grid), dim3(256), 0, s, p);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = temp_bytes;
    return rocprim::radix_sort_pairs<HistSortConfig>(temp, tb, (const uint32_t*)p.keys, hist_slot, (const uint8_t*)p.vals, hist,
                                     (size_t)p.n_slots, 0u, key_bits(p.sentinel), s);
}

}  // namespace fbk
