// fb_hist.hip -- per-flow history characters of one flow-table update, in packet order.
//
// The reference appends map_tcp_flags(..) to the flow's `history` String for every TCP packet
// (src/packets.rs:187-198 occupied, 410-426 vacant), so a flow's history is its TCP packets'
// characters in arrival order.  fb_flow_history_dev returns the last update's characters grouped
// per flow: a stable sort of its TCP records by table slot.  No global sort is needed: the update
// already bucketed every record by table partition (= slot / 512), and k_flow_apply left one
// history word per entry it applied (slot in the partition | character code | record within its
// bucketing chunk), each partition's words contiguous and in chunk (= record) order:
//   k_hist_scan : exclusive scan of the per-partition character counts k_flow_apply reported
//                 (partials[4 p + 3]) -> each partition's output offset; the total -> *n_hist.
//   k_hist_uniform : one workgroup per partition, for a partition of one chunk round, at most
//                 kHistCap entries, no combined group and no chunk run over kRunSort entries (the
//                 uniform case; the others are listed for k_hist_general):
//                 1. thread t sorts chunk run t by record in registers (K1's scatter leaves a run
//                    unordered) into LDS at the run's place: the partition is then in record order;
//                 2. per wave and slot, the characters counted (LDS atomics); per slot, a scan over
//                    the waves from the slot's offset (hcount scanned);
//                 3. the walk: wave w takes its 64 runs, 64 entries a step: a key's output position
//                    = its wave's position for the slot + the slot's lanes below it in the step;
//                    the lowest lane moves it on.  Stable by record without a comparison sort; the
//                    output is staged in LDS and written coalesced.
//   k_hist_general : the listed partitions, a grid-stride loop: chunk rounds of 512 runs, batches
//                 of at most kHistCap entries, each put in record order and walked as above.  A
//                 run k_flow_combine folded (a hot group) is read from e_sort, which K1c wrote in
//                 record order (the original entry word, and the record's slot through its
//                 combined entry's agg_slot or its moved entry's history word); a plain run of
//                 more than kRunSort entries is sorted by a wavefront or, past kWaveSortMax, by a
//                 bitmap of the chunk's records.  A partition with many entries or characters (a
//                 skewed batch) is split over chunk blocks: k_hist_general<true> counts each
//                 block's characters per slot, k_hist_blocks scans them over the blocks, and each
//                 block starts its slots after the earlier blocks'.
// Bytes per entry: its 4-B history word (8-B e_sort word) read; per character 5 B written (+ the
// count arrays).
#include "fb_internal.h"

namespace fbk {

constexpr uint32_t kHistThreads = 512;
#ifndef FB_HIST_CAP
#define FB_HIST_CAP 4096
#endif
constexpr uint32_t kHistCap = FB_HIST_CAP;  // entries per batch (8 B of LDS each)
constexpr uint32_t kHistRuns = 512;         // chunk runs per round: one per thread
constexpr uint32_t kRunSort = 16;           // (uniform) the longest chunk run sorted in registers
constexpr uint32_t kHistWaves = kHistThreads / 64;
constexpr uint32_t kHistPer = kHistCap / kHistThreads;
static_assert(kFlowSlots == kHistThreads && kHistRuns == kHistThreads, "one slot / run per thread");
static_assert(kHistWaves * kFlowSlots <= kHistCap, "the waves' slot counts share the keys' LDS");

// History character of a code (1 + FB_HIST_CHARS index) from two packed constants: no table load.
__device__ __forceinline__ uint8_t hist_char_of(uint32_t code) {
    constexpr unsigned long long kLo = 0x5266466848735300ull;  // "\0SsHhFfR", byte k = code k
    constexpr unsigned long long kHi = 0x2D61413C3E72ull;    // "r><Aa-", byte k = code 8 + k
    return (uint8_t)(((code < 8u) ? kLo : kHi) >> (8u * (code & 7u)));
}

// Ascending bitonic network over a[0 .. N) (registers: every index is a constant once unrolled).
template <int N>
__device__ __forceinline__ void sort_net(uint32_t (&a)[kRunSort]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const uint32_t x = a[i], y = a[l], lo = min(x, y), hi = max(x, y);
                    const bool up = (i & k) == 0;
                    a[i] = up ? lo : hi;
                    a[l] = up ? hi : lo;
                }
            }
        }
    }
}

__device__ __forceinline__ uint32_t block_scan2(uint32_t v, uint32_t v2, uint32_t& tot, uint32_t& ex2, uint32_t& tot2,
                                                uint32_t* wsum, uint32_t* wsum2) {
    // block-wide exclusive sums of two values per thread (blockDim.x / 64 <= 16 waves)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v, x2 = v2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64), y2 = __shfl_up(x2, o, 64);
        if (lane >= (uint32_t)o) {
            x += y;
            x2 += y2;
        }
    }
    if (lane == 63u) {
        wsum[wave] = x;
        wsum2[wave] = x2;
    }
    __syncthreads();
    uint32_t before = 0u, before2 = 0u;
    tot = tot2 = 0u;
    for (uint32_t k = 0; k < nw; ++k) {
        const uint32_t s = wsum[k], s2 = wsum2[k];
        if (k < wave) {
            before += s;
            before2 += s2;
        }
        tot += s;
        tot2 += s2;
    }
    __syncthreads();
    ex2 = before2 + x2 - v2;
    return before + x - v;
}

// Exclusive scan of the partitions' character counts (partials[4 p + 3] low word) -> part_base;
// one pass: thread t sums a contiguous group of partitions, one block scan, the group written.
__global__ __launch_bounds__(1024) void k_hist_scan(const unsigned long long* partials, uint32_t parts,
                                                    uint32_t* part_base, uint32_t* n_hist, uint32_t* slow,
                                                    uint32_t* hot) {
    __shared__ uint32_t wsum[16], wsum2[16];
    const uint32_t per = (parts + 1023u) / 1024u, p0 = min(threadIdx.x * per, parts), p1 = min(p0 + per, parts);
    uint32_t sum = 0u;
    for (uint32_t i = p0; i < p1; ++i) sum += (uint32_t)partials[4 * (size_t)i + 3];
    uint32_t tot, ex2, tot2;
    uint32_t run = block_scan2(sum, 0u, tot, ex2, tot2, wsum, wsum2);
    for (uint32_t i = p0; i < p1; ++i) {
        part_base[i] = run;
        run += (uint32_t)partials[4 * (size_t)i + 3];
    }
    if (threadIdx.x == 0) {
        part_base[parts] = tot;
        *n_hist = tot;
        slow[0] = 0u;  // k_hist_uniform lists the partitions it leaves to k_hist_general
        if (hot) hot[0] = 0u;
    }
}

// A listed partition with more than kHistSplitEntries entries to read (a combined group's: its
// records) goes to a second list (up to kHistListCap) and is split by chunk blocks of about
// kHistBlockEntries entries: k_hist_general<true> counts each block's characters per slot into
// cnt[list index][block][slot], k_hist_blocks scans them over the blocks, and each block's
// k_hist_general<false> workgroup starts its slots' cursors there.  Skewed batches need it: under
// Zipf(1.1) one workgroup spent 25 ms on the hottest flow's partition (~12 % of the records) and
// ~1.5 ms on one of 42K entries (a flow with ~0.4 %).  A C4 partition holds ~2,560 entries.
#ifndef FB_HIST_SPLIT_ENTRIES
#define FB_HIST_SPLIT_ENTRIES 8192
#endif
constexpr uint32_t kHistSplitEntries = FB_HIST_SPLIT_ENTRIES;
#ifndef FB_HIST_BLOCK_ENTRIES
#define FB_HIST_BLOCK_ENTRIES 4096
#endif
constexpr uint32_t kHistBlockEntries = FB_HIST_BLOCK_ENTRIES;
constexpr uint32_t kHistListCap = 256;    // split partitions (cnt rows)
constexpr uint32_t kHistMaxBlocks = 128;  // chunk blocks of at least kHistBlockChunks chunks
constexpr uint32_t kHistBlockChunks = 4;
constexpr uint32_t kHistSplitGrid = 2048;  // workgroups over the split partitions' (partition, block) pairs

// ---- the uniform case: one chunk round, <= kHistCap entries, every run <= kRunSort plain entries,
// every wave's share (its 64 runs) <= kHistPer steps of 64
struct UniLds {
    uint32_t skeys[kHistCap];                // run-sorted keys, then the output stage
    uint32_t hist[kHistWaves * kFlowSlots];  // [wave][slot]: count, then next output position
    uint32_t rn[kHistRuns];                  // run lengths (bit 31: combined) } the walk's slot tags
    uint32_t rq[kHistRuns];                  // first history word of a run      } (u8 [wave][slot])
    uint32_t rp[kHistRuns + 1];              // exclusive prefix of rn
    uint32_t wsum[kHistWaves], wsum2[kHistWaves];
};
static_assert(sizeof(UniLds) <= 40u * 1024u, "four workgroups per CU");

__global__ __launch_bounds__(kHistThreads) void k_hist_uniform(const FlowParams P, uint32_t chunks, uint32_t* out_slot,
                                                               uint8_t* out_char, uint32_t* slow, uint32_t* hot) {
    __shared__ UniLds L;
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // every load issued together: the partition's character count and history-word base, its
    // output offset, its slots' counts, its chunk runs
    const unsigned long long pw = P.partials[4 * (size_t)q + 3];
    const uint32_t out_beg = P.part_base[q];
    const uint32_t hc = P.hcount[(size_t)q * kFlowSlots + tid];
    const uint32_t vp = tid < chunks ? P.cols[(size_t)q * P.chunk_stride + tid] : 0u;
    const uint32_t n_chars = (uint32_t)pw, hbase = (uint32_t)(pw >> 32);
    if (n_chars == 0u) return;  // uniform: no history characters in this partition
    for (uint32_t j = tid; j < kHistWaves * kFlowSlots; j += kHistThreads) L.hist[j] = 0u;
    const bool comb = (vp & 0x8000u) != 0u;
    const uint32_t lp = vp >> 16, len = comb ? 0x80000000u : lp;  // (combined: the general kernel's)
    uint32_t tp, ep, tc;
    // run offsets (entries) and the slots' first output positions, one pair of barriers
    const uint32_t cur = block_scan2(hc, lp, tc, ep, tp, L.wsum, L.wsum2);  // slot tid's first position
    L.rp[tid] = ep;
    if (tid == 0) L.rp[kHistRuns] = tp;
    __syncthreads();
    const uint32_t wlen = L.rp[min(64u * wave + 64u, kHistRuns)] - L.rp[64u * wave];
    if (__syncthreads_or(len > kRunSort || wlen > kHistPer * 64u) || chunks > kHistRuns || tp > kHistCap) {
        // uniform: the general kernels take it; a partition with many characters or entries to read
        // (a combined group's: its original row) is split
        uint32_t rd = 0u, tr, ex2, tot2;
        for (uint32_t c = tid; hot && c < chunks; c += kHistThreads) {
            const uint32_t v = P.cols[(size_t)q * P.chunk_stride + c];
            rd += (v & 0x8000u) ? P.rows_h[(size_t)c * P.parts + q] >> 16 : v >> 16;
        }
        block_scan2(rd, 0u, tr, ex2, tot2, L.wsum, L.wsum2);
        if (tid == 0) {
            uint32_t h = ~0u;
            if (hot && tr > kHistSplitEntries) h = atomicAdd(hot, 1u);
            // the split list entry: partition | blocks wanted << 16 (k_hist_general caps them)
            if (h < kHistListCap) hot[1u + h] = q | min((tr + kHistBlockEntries - 1u) / kHistBlockEntries, 0xFFFFu) << 16;
            else slow[1u + atomicAdd(slow, 1u)] = q;
        }
        return;
    }
    {   // run tid in record order (K1's scatter leaves a run unordered): key = record in chunk << 13
        // | slot << 4 | code; the wave's slot counts by LDS atomics (order-free)
        uint32_t a[kRunSort];
        const __amdgpu_buffer_rsrc_t rh =
            __builtin_amdgcn_make_buffer_rsrc((void*)P.hword, (short)0, (int)(P.max_recs * 4u), 0x00020000);
        const uint32_t vo = (hbase + ep) * 4u;
#pragma unroll
        for (uint32_t k = 0; k < kRunSort; ++k)  // unpredicated: all in flight, past-run words masked
            a[k] = __builtin_amdgcn_raw_buffer_load_b32(rh, vo + 4u * k, 0, 0);
        uint32_t* hw = L.hist + wave * kFlowSlots;
#pragma unroll
        for (uint32_t k = 0; k < kRunSort; ++k) {
            const uint32_t w = a[k];
            a[k] = k < len ? (w >> 13) << 13 | (w & 0x1FFu) << 4 | ((w >> 9) & 15u) : ~0u;
            if (k < len && ((w >> 9) & 15u)) atomicAdd(hw + (w & 0x1FFu), 1u);
        }
        uint32_t wl = len;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o, 64));
        if (wl > 8u) sort_net<16>(a);
        else if (wl > 4u) sort_net<8>(a);
        else if (wl > 1u) sort_net<4>(a);
#pragma unroll
        for (uint32_t k = 0; k < kRunSort; ++k)
            if (k < len) L.skeys[ep + k] = a[k];
    }
    __syncthreads();
    {   // per slot: each wave's first output position = the slot's + the earlier waves' counts
        uint32_t run = cur;
#pragma unroll
        for (uint32_t w = 0; w < kHistWaves; ++w) {
            const uint32_t x = L.hist[w * kFlowSlots + tid];
            L.hist[w * kFlowSlots + tid] = run;
            run += x;
        }
    }
    __syncthreads();
    // the wave's entries (its 64 runs) in order, 64 a step: a key's position = its wave's next one
    // for the slot + the step's lanes below it holding the slot; the lowest such lane moves it on.
    // Lanes sharing a slot find each other through a tag per slot: each TCP lane writes its lane
    // number and reads it back; a lane finding another number shares its slot, and only those
    // slots (a few per step) take a ballot each.
    const uint32_t lo_w = L.rp[64u * wave], hi_w = L.rp[min(64u * wave + 64u, kHistRuns)];
    uint32_t* hw = L.hist + wave * kFlowSlots;
    uint8_t* tag = reinterpret_cast<uint8_t*>(L.rn) + wave * kFlowSlots;
    static_assert(sizeof(L.rn) + sizeof(L.rq) == kHistWaves * kFlowSlots, "tags fill rn and rq");
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t dst[kHistPer], val[kHistPer];
#pragma unroll
    for (uint32_t s = 0; s < kHistPer; ++s) {
        const uint32_t e = lo_w + s * 64u + lane;
        dst[s] = ~0u;
        val[s] = 0u;
        if (lo_w + s * 64u >= hi_w) continue;  // wave-uniform
        const uint32_t key = e < hi_w ? L.skeys[e] : 0u, sl = (key >> 4) & 511u;
        const bool tcp = e < hi_w && (key & 15u) != 0u;
        if (tcp) tag[sl] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();
        unsigned long long pending = __ballot(tcp && tag[sl] != lane), m = 1ull << lane;
        while (pending) {  // wave-uniform
            const uint32_t l = (uint32_t)__builtin_ctzll(pending);
            const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)sl, (int)l);
            const unsigned long long pm = __ballot(tcp && sl == o);
            if (tcp && sl == o) m = pm;
            pending &= ~pm;
        }
        if (tcp) {
            dst[s] = hw[sl] + (uint32_t)__popcll(m & below);
            val[s] = sl | (uint32_t)hist_char_of(key & 15u) << 16;
        }
        __builtin_amdgcn_wave_barrier();
        if (tcp && (m & below) == 0ull) hw[sl] += (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();  // every key read: stage the output in its order, one coalesced write
#pragma unroll
    for (uint32_t s = 0; s < kHistPer; ++s)
        if (dst[s] < n_chars) L.skeys[dst[s]] = val[s];
    __syncthreads();
    for (uint32_t i = tid; i < n_chars; i += kHistThreads) {
        const uint32_t v = L.skeys[i];
        out_slot[out_beg + i] = q * kFlowSlots + (v & 0xFFFFu);
        out_char[out_beg + i] = (uint8_t)(v >> 16);
    }
}

constexpr uint32_t kBmWords = kFlowChunk / 32u;  // a chunk's records as a bitmap (640 words)
struct HistLds {
    uint32_t skey[kHistCap];                 // the batch's keys in entry order: record in chunk << 13 |
                                             // slot << 4 | code, ~0 for no character
    uint32_t skey2[kHistCap];                // the same with every run sorted by record
    uint32_t wcnt[kHistWaves * kFlowSlots];  // the walk: [wave][slot] counts, then output positions
    uint8_t tag[kHistWaves * kFlowSlots];    // the walk's slot tags
    uint32_t bm[kBmWords], bmp[kBmWords];    // a long run's records as a bitmap, prefix popcounts
    uint32_t cursor[kFlowSlots], bcnt[kFlowSlots];
    uint32_t rs[kHistRuns];      // run r (chunk c0 + r): its first entry position
    uint32_t rn[kHistRuns];      // its entries to read (bit 31: a combined group, e_sort)
    uint32_t rp[kHistRuns + 1];  // exclusive prefix of rn
    uint32_t rq[kHistRuns];      // the history word of its first applied entry
    uint32_t lst[kHistRuns];     // the batch's runs of more than 64 entries (then of 17..64: from the back)
    uint32_t wsum[kHistThreads / 64], wsum2[kHistThreads / 64];
    uint32_t pairs[kHistListCap + 1];  // (split) exclusive prefix of the listed partitions' blocks
    uint32_t s_n, s_m;
};
static_assert(sizeof(HistLds) <= 80u * 1024u, "two workgroups per CU");

// Listed partitions: `slow` (one workgroup each, every chunk) and `hot`, the split partitions (with
// nblk > 1; cnt = their [list index][block][slot] counts) -- a grid-stride loop over the pairs.
// Slot (within the partition) of a record of a combined group: its combined entry's agg_slot, or the
// history word of its moved plain entry.  An entry the table could not take (partition full / spin
// expired: error bit 4 / 16) left agg_slot ~0 or history word 0 -- its character is dropped (code 0)
// instead of being filed under a slot some other flow holds.
__device__ __forceinline__ uint32_t combined_slot(const FlowParams& P, uint32_t m, uint32_t rq, uint32_t rs,
                                                  uint32_t& code) {
    const bool comb = (m & kRecFlowCombined) != 0u;
    const uint32_t v = comb ? P.agg_slot[m & ~kRecFlowCombined] : P.hword[rq + (m - rs)];
    if (comb ? v == ~0u : v == 0u) code = 0u;
    return v & (kFlowSlots - 1u);
}

// One plain run of 17 .. 64 K keys placed in record order by a wavefront: lane l holds keys l, l + 64 ..
// (K per lane); a key's place = the run's keys below it (keys are distinct records, read from LDS
// four at a time, the same address in every lane: broadcasts); ~0 (no character) keys go after the
// others, in lane order.  src -> dst (LDS).  (A bitonic network over the lanes spent a dependent
// cross-lane permute per step: ~20 per 64 keys.)
constexpr uint32_t kWaveSortMax = 512;  // longer runs: the block's bitmap rank
template <uint32_t K>
__device__ __forceinline__ void wave_sort_run(const uint32_t* src, uint32_t* dst, uint32_t len, uint32_t lane) {
    uint32_t x[K], rank[K];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) {
        x[j] = j * 64u + lane < len ? src[j * 64u + lane] : ~0u;
        rank[j] = 0u;
    }
    const uint32_t len4 = len & ~3u;
    for (uint32_t i = 0; i < len4; i += 4u) {  // (src is 4-B aligned only: four scalar-address reads)
        const uint32_t y0 = src[i], y1 = src[i + 1u], y2 = src[i + 2u], y3 = src[i + 3u];
#pragma unroll
        for (uint32_t j = 0; j < K; ++j)
            rank[j] += (uint32_t)(y0 < x[j]) + (uint32_t)(y1 < x[j]) + (uint32_t)(y2 < x[j]) + (uint32_t)(y3 < x[j]);
    }
    for (uint32_t i = len4; i < len; ++i) {
        const uint32_t y = src[i];
#pragma unroll
        for (uint32_t j = 0; j < K; ++j) rank[j] += (uint32_t)(y < x[j]);
    }
    // the ~0 keys: after the n_tcp others, in (register, lane) order
    uint32_t none_before = 0u;
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) {
        const bool in = j * 64u + lane < len, none = in && x[j] == ~0u;
        const unsigned long long m = __ballot(none);
        if (none) rank[j] += none_before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        none_before += (uint32_t)__popcll(m);
        // (a ~0 key counted the run's other keys below ~0, i.e. every TCP key: its base is n_tcp)
    }
#pragma unroll
    for (uint32_t j = 0; j < K; ++j)
        if (j * 64u + lane < len) dst[rank[j]] = x[j];
}

template <bool COUNT>
__global__ __launch_bounds__(kHistThreads, 4) void k_hist_general(const FlowParams P, uint32_t chunks, uint32_t* out_slot,
                                                               uint8_t* out_char, const uint32_t* slow,
                                                               const uint32_t* hot, uint32_t* cnt, uint32_t nblk) {
    __shared__ HistLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    // block-wide exclusive sums of one or two values per thread (tot: the sum)
    auto block_scan2 = [&](uint32_t v, uint32_t v2, uint32_t& tot, uint32_t& ex2, uint32_t& tot2) {
        uint32_t x = v, x2 = v2;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64), y2 = __shfl_up(x2, o, 64);
            if (lane >= (uint32_t)o) {
                x += y;
                x2 += y2;
            }
        }
        if (lane == 63u) {
            L.wsum[wave] = x;
            L.wsum2[wave] = x2;
        }
        __syncthreads();
        uint32_t before = 0u, before2 = 0u;
        tot = tot2 = 0u;
        for (uint32_t k = 0; k < kHistThreads / 64u; ++k) {
            const uint32_t s = L.wsum[k], s2 = L.wsum2[k];
            if (k < wave) {
                before += s;
                before2 += s2;
            }
            tot += s;
            tot2 += s2;
        }
        __syncthreads();
        ex2 = before2 + x2 - v2;
        return before + x - v;
    };
    auto block_scan = [&](uint32_t v, uint32_t& tot) {
        uint32_t ex2, tot2;
        return block_scan2(v, 0u, tot, ex2, tot2);
    };

    auto partition = [&](uint32_t q, uint32_t li, uint32_t blk, uint32_t nb) {
        // every load the first round needs, issued together: the partition's character count and
        // history-word base, its output range, its slots' counts
        const unsigned long long pw = P.partials[4 * (size_t)q + 3];
        const uint32_t out_beg = P.part_base[q], out_end = P.part_base[q + 1];
        const uint32_t hc = P.hcount[(size_t)q * kFlowSlots + tid];
        const uint32_t* col = P.cols + (size_t)q * P.chunk_stride;
        const uint32_t n_chars = (uint32_t)pw, hbase = (uint32_t)(pw >> 32);
        if (n_chars == 0u) return;  // uniform: no history characters in this partition
        // this workgroup's chunk block (a partition that is not split: every chunk)
        const bool split = nb > 1u;  // (nb blocks of this partition, <= nblk)
        const uint32_t cbs = split ? (chunks + nb - 1u) / nb : chunks;
        const uint32_t cb0 = blk * cbs, cb1 = min(chunks, cb0 + cbs);
        if (cb0 >= cb1) return;  // uniform
        uint32_t vp = tid < cb1 - cb0 ? col[cb0 + tid] : 0u;
        uint32_t before = 0u;  // applied entries (history words) of the chunks before the block
        for (uint32_t c = tid; c < cb0; c += kHistThreads) before += col[c] >> 16;
        uint32_t* bc = cnt + ((size_t)li * nblk) * kFlowSlots;  // (split) [block][slot] counts
        {
            uint32_t t;
            // the slot's characters in the earlier blocks (k_hist_blocks' prefix)
            const uint32_t prior = (!COUNT && split) ? bc[(size_t)blk * kFlowSlots + tid] : 0u;
            L.cursor[tid] = block_scan(hc, t) + prior;  // relative to out_beg
            L.bcnt[tid] = 0u;
            uint32_t tb;
            block_scan(before, tb);
            before = tb;
        }
        uint32_t carry = hbase + before;  // history word of the round's first applied entry
        // round setup: the runs of chunks c0 .. c0 + 511 (tid: run tid); returns the entries read
        auto round = [&](uint32_t c0, uint32_t nr) {
            const uint32_t c = c0 + tid;
            const bool comb = tid < nr && (vp & 0x8000u) != 0u;
            // a combined group's original row (its records in e_sort): rows_h, read only for those
            const uint32_t vh = comb ? P.rows_h[(size_t)c * P.parts + q] : 0u;
            const uint32_t lp = tid < nr ? vp >> 16 : 0u, lv = comb ? vh >> 16 : lp;  // applied / read entries
            L.rs[tid] = c * kFlowChunk + (vp & 0x7FFFu);  // (k_flow_combine packs a group in place)
            L.rn[tid] = lv | (comb ? 1u << 31 : 0u);
            uint32_t tv, tp, ep;
            const uint32_t ev = block_scan2(lv, lp, tv, ep, tp);
            L.rp[tid] = ev;
            L.rq[tid] = carry + ep;
            if (tid == 0) L.rp[kHistRuns] = tv;
            carry += tp;
            __syncthreads();
            return tv;
        };
        const uint32_t nr0 = min(kHistRuns, cb1 - cb0);
        const uint32_t tv0 = round(cb0, nr0);
        if constexpr (COUNT) {  // this block's characters per slot
            for (uint32_t c0 = cb0; c0 < cb1; c0 += kHistRuns) {
                const uint32_t nr = min(kHistRuns, cb1 - c0);
                if (c0 != cb0) {
                    vp = tid < nr ? col[c0 + tid] : 0u;
                    round(c0, nr);
                }
                const uint32_t tv = L.rp[nr];
                for (uint32_t e = tid; e < tv; e += kHistThreads) {
                    uint32_t lo = 0u, hi = nr - 1u;  // the run holding e
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi + 1u) >> 1;
                        if (L.rp[mid] <= e) lo = mid; else hi = mid - 1u;
                    }
                    const uint32_t k = e - L.rp[lo];
                    uint32_t slot = 0u, code;
                    if (!(L.rn[lo] >> 31)) {
                        const uint32_t w = P.hword[L.rq[lo] + k];
                        slot = w & (kFlowSlots - 1u);
                        code = (w >> 9) & 15u;
                    } else {
                        const uint2 es = P.e_sort[L.rs[lo] + k];
                        code = (es.x >> kEntCodeShift) & 15u;
                        if (code != 0u) slot = combined_slot(P, es.y, L.rq[lo], L.rs[lo], code);
                    }
                    if (code != 0u) atomicAdd(&L.bcnt[slot], 1u);
                }
                __syncthreads();
            }
            bc[(size_t)blk * kFlowSlots + tid] = L.bcnt[tid];
            return;
        } else {
            // Output order per slot = record order.  A batch of whole runs (<= kHistCap entries, runs
            // in chunk order) is loaded as 32-bit keys (record in chunk << 13 | slot << 4 | code),
            // each run sorted by record -- K1's scatter leaves a run unordered: runs of <= 16 entries
            // by their thread in registers, <= 64 by a wavefront (bitonic over the lanes), longer ones
            // block-wide by a bitmap of the chunk's records (rank = the set bits below) -- so the
            // batch is in record order; the walk then hands each character its slot's next output
            // position (per-wave slot counts, a scan per slot, the k_hist_uniform walk).  No
            // comparison sort of a whole batch: a skewed batch (one slot with most of its keys)
            // costs what a uniform one does.
            auto run_of = [&](uint32_t e, uint32_t r0, uint32_t r1) {  // the largest r with rp[r] <= e
                uint32_t lo = r0, hi = r1 - 1u;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1u) >> 1;
                    if (L.rp[mid] <= e) lo = mid; else hi = mid - 1u;
                }
                return lo;
            };
            auto key_of = [&](uint32_t e, uint32_t r, uint32_t c0) {  // round entry e of run r
                const uint32_t k = e - L.rp[r];
                uint32_t slot = 0u, code, rec;
                if (!(L.rn[r] >> 31)) {
                    const uint32_t w = P.hword[L.rq[r] + k];
                    slot = w & (kFlowSlots - 1u);
                    code = (w >> 9) & 15u;
                    rec = w >> 13;  // (record % kFlowChunk)
                } else {
                    const uint2 es = P.e_sort[L.rs[r] + k];
                    code = (es.x >> kEntCodeShift) & 15u;
                    rec = (es.x & kEntRecMask) - (c0 + r) * kFlowChunk;
                    if (code != 0u) slot = combined_slot(P, es.y, L.rq[r], L.rs[r], code);
                }
                return code != 0u ? rec << 13 | slot << 4 | code : ~0u;
            };
            auto emit = [&](uint32_t dst, uint32_t key) {
                dst += out_beg;
                if (dst < out_end) {  // (a table-full batch may hold fewer slot counts than characters)
                    out_slot[dst] = q * kFlowSlots + ((key >> 4) & (kFlowSlots - 1u));
                    out_char[dst] = hist_char_of(key & 15u);
                }
            };
            // block-wide exclusive scan of the bitmap's popcounts (nw <= kBmWords words)
            auto bitmap_prefix = [&](uint32_t nw) {
                const uint32_t w0 = 2u * tid, c0w = w0 < nw ? __popc(L.bm[w0]) : 0u,
                               c1w = w0 + 1u < nw ? __popc(L.bm[w0 + 1u]) : 0u;
                uint32_t tot;
                const uint32_t ex = block_scan(c0w + c1w, tot);
                if (w0 < nw) L.bmp[w0] = ex;
                if (w0 + 1u < nw) L.bmp[w0 + 1u] = ex + c0w;
                __syncthreads();
                return tot;
            };
            auto rank_of = [&](uint32_t rec) {
                const uint32_t w = rec >> 5;
                return L.bmp[w] + __popc(L.bm[w] & ((1u << (rec & 31u)) - 1u));
            };
            static_assert(2u * kHistThreads >= kBmWords, "two bitmap words per thread");
            // the walk over skey2[0 .. n): stable per slot, output positions from the slots' cursors
            auto walk = [&](uint32_t n) {
                const uint32_t span = ((n + kHistThreads - 1u) / kHistThreads) * 64u;
                const uint32_t lo_w = min(wave * span, n), hi_w = min(lo_w + span, n);
                uint32_t* hw = L.wcnt + wave * kFlowSlots;
                for (uint32_t i = lo_w + lane; i < hi_w; i += 64u) {
                    const uint32_t k = L.skey2[i];
                    if (k != ~0u) atomicAdd(hw + ((k >> 4) & (kFlowSlots - 1u)), 1u);
                }
                __syncthreads();
                {   // slot tid: each wave's first position = the cursor + the earlier waves' counts
                    uint32_t run = L.cursor[tid];
#pragma unroll
                    for (uint32_t w = 0; w < kHistWaves; ++w) {
                        const uint32_t x = L.wcnt[w * kFlowSlots + tid];
                        L.wcnt[w * kFlowSlots + tid] = run;
                        run += x;
                    }
                    L.cursor[tid] = run;
                }
                __syncthreads();
                uint8_t* tg = L.tag + wave * kFlowSlots;
                const unsigned long long below = (1ull << lane) - 1ull;
                for (uint32_t b0 = lo_w; b0 < hi_w; b0 += 64u) {  // wave-uniform
                    const uint32_t i = b0 + lane;
                    const uint32_t k = i < hi_w ? L.skey2[i] : ~0u;
                    const bool tcp = k != ~0u;
                    const uint32_t sl = (k >> 4) & (kFlowSlots - 1u);
                    if (tcp) tg[sl] = (uint8_t)lane;
                    __builtin_amdgcn_wave_barrier();
                    unsigned long long pending = __ballot(tcp && tg[sl] != lane), m = 1ull << lane;
                    while (pending) {  // the few slots several lanes hold: one ballot each
                        const uint32_t l = (uint32_t)__builtin_ctzll(pending);
                        const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)sl, (int)l);
                        const unsigned long long pm = __ballot(tcp && sl == o);
                        if (tcp && sl == o) m = pm;
                        pending &= ~pm;
                    }
                    if (tcp) emit(hw[sl] + (uint32_t)__popcll(m & below), k);
                    __builtin_amdgcn_wave_barrier();
                    if (tcp && (m & below) == 0ull) hw[sl] += (uint32_t)__popcll(m);
                    __builtin_amdgcn_wave_barrier();
                }
                __syncthreads();
                for (uint32_t j = tid; j < kHistWaves * kFlowSlots; j += kHistThreads) L.wcnt[j] = 0u;
                // (the next writer of wcnt is past a barrier)
            };
            for (uint32_t j = tid; j < kHistWaves * kFlowSlots; j += kHistThreads) L.wcnt[j] = 0u;
            // entries [e0, e1) (<= kHistCap) of runs r0 .. r1 - 1
            auto batch = [&](uint32_t r0, uint32_t r1, uint32_t e0, uint32_t e1, uint32_t c0) {
                const uint32_t n = e1 - e0;
                if (tid == 0) {
                    L.s_n = 0u;
                    L.s_m = 0u;
                }
                // the keys, kLoadGroup per thread with their loads in flight together: each entry's
                // run (binary search in LDS), its history word or (a combined group) its e_sort
                // word; then the combined records' slots (agg_slot / the moved entry's history word)
                constexpr uint32_t kLoadGroup = 4;
                for (uint32_t g0 = 0; g0 < kHistPer; g0 += kLoadGroup) {
                    uint32_t rr[kLoadGroup], w1[kLoadGroup], m1[kLoadGroup], w2[kLoadGroup];
#pragma unroll
                    for (uint32_t u = 0; u < kLoadGroup; ++u) {
                        const uint32_t i = tid + (g0 + u) * kHistThreads;
                        rr[u] = i < n ? run_of(e0 + i, r0, r1) : r0;
                    }
#pragma unroll
                    for (uint32_t u = 0; u < kLoadGroup; ++u) {
                        const uint32_t i = tid + (g0 + u) * kHistThreads, r = rr[u];
                        const uint32_t k = e0 + i - L.rp[r];
                        const bool comb = (L.rn[r] >> 31) != 0u;
                        if (i < n && comb) {
                            const uint2 es = P.e_sort[L.rs[r] + k];
                            w1[u] = es.x;
                            m1[u] = es.y;
                        } else {
                            w1[u] = i < n ? P.hword[L.rq[r] + k] : 0u;
                            m1[u] = 0u;
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < kLoadGroup; ++u) {
                        const uint32_t i = tid + (g0 + u) * kHistThreads, r = rr[u];
                        const bool need = i < n && (L.rn[r] >> 31) != 0u && ((w1[u] >> kEntCodeShift) & 15u) != 0u;
                        const uint32_t m = m1[u];
                        w2[u] = !need ? 0u : (m & kRecFlowCombined) ? P.agg_slot[m & ~kRecFlowCombined]
                                                                      : P.hword[L.rq[r] + (m - L.rs[r])];
                    }
#pragma unroll
                    for (uint32_t u = 0; u < kLoadGroup; ++u) {
                        const uint32_t i = tid + (g0 + u) * kHistThreads, r = rr[u];
                        if (i >= n) continue;
                        uint32_t slot, code, rec;
                        if (!(L.rn[r] >> 31)) {
                            slot = w1[u] & (kFlowSlots - 1u);
                            code = (w1[u] >> 9) & 15u;
                            rec = w1[u] >> 13;
                        } else {
                            code = (w1[u] >> kEntCodeShift) & 15u;
                            rec = (w1[u] & kEntRecMask) - (c0 + r) * kFlowChunk;
                            // an entry the table could not take: agg_slot ~0 / history word 0 (combined_slot)
                            if ((m1[u] & kRecFlowCombined) ? w2[u] == ~0u : w2[u] == 0u) code = 0u;
                            slot = w2[u] & (kFlowSlots - 1u);
                        }
                        // a combined run (e_sort) is in record order already: straight to skey2
                        (L.rn[r] >> 31 ? L.skey2 : L.skey)[i] = code != 0u ? rec << 13 | slot << 4 | code : ~0u;
                    }
                }
                __syncthreads();
                {   // plain runs of <= kRunSort entries: their thread, in registers; the others listed
                    // -- up to kWaveSortMax entries for a wavefront (front of lst), longer ones for
                    // the whole block (back of lst)
                    const uint32_t r = r0 + tid;
                    const bool plain = r < r1 && !(L.rn[r] >> 31);
                    const uint32_t b = plain ? L.rp[r] - e0 : 0u, len = plain ? L.rp[r + 1u] - L.rp[r] : 0u;
                    if (len > kWaveSortMax) L.lst[kHistRuns - 1u - atomicAdd(&L.s_n, 1u)] = r;
                    else if (len > kRunSort) L.lst[atomicAdd(&L.s_m, 1u)] = r;
                    uint32_t a[kRunSort];
#pragma unroll
                    for (uint32_t k = 0; k < kRunSort; ++k) a[k] = (len <= kRunSort && k < len) ? L.skey[b + k] : ~0u;
                    uint32_t wl = len <= kRunSort ? len : 0u;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o, 64));
                    if (wl > 8u) sort_net<16>(a);
                    else if (wl > 4u) sort_net<8>(a);
                    else if (wl > 1u) sort_net<4>(a);
#pragma unroll
                    for (uint32_t k = 0; k < kRunSort; ++k)
                        if (len <= kRunSort && k < len) L.skey2[b + k] = a[k];
                }
                __syncthreads();
                // plain runs of 17 .. kWaveSortMax entries: a wavefront each, 1 / 2 / 4 / 8 keys a lane
                for (uint32_t j = wave; j < L.s_m; j += kHistWaves) {
                    const uint32_t r = L.lst[j];
                    const uint32_t b = L.rp[r] - e0, len = L.rp[r + 1u] - L.rp[r];
                    if (len <= 64u) wave_sort_run<1>(L.skey + b, L.skey2 + b, len, lane);
                    else if (len <= 128u) wave_sort_run<2>(L.skey + b, L.skey2 + b, len, lane);
                    else if (len <= 256u) wave_sort_run<4>(L.skey + b, L.skey2 + b, len, lane);
                    else wave_sort_run<8>(L.skey + b, L.skey2 + b, len, lane);
                }
                // longer runs: block-wide, one at a time, ranked by the bitmap of the chunk's records
                const uint32_t nl = L.s_n;
                for (uint32_t j = 0; j < nl; ++j) {  // uniform
                    const uint32_t r = L.lst[kHistRuns - 1u - j];
                    const uint32_t b = L.rp[r] - e0, len = L.rp[r + 1u] - L.rp[r];
                    for (uint32_t w = tid; w < kBmWords; w += kHistThreads) L.bm[w] = 0u;
                    for (uint32_t i = tid; i < len; i += kHistThreads) L.skey2[b + i] = ~0u;
                    __syncthreads();
                    for (uint32_t i = tid; i < len; i += kHistThreads) {
                        const uint32_t k = L.skey[b + i];
                        if (k != ~0u) atomicOr(&L.bm[k >> 18], 1u << ((k >> 13) & 31u));
                    }
                    __syncthreads();
                    bitmap_prefix(kBmWords);
                    for (uint32_t i = tid; i < len; i += kHistThreads) {
                        const uint32_t k = L.skey[b + i];
                        if (k != ~0u) L.skey2[b + rank_of(k >> 13)] = k;
                    }
                    __syncthreads();
                }
                __syncthreads();
                walk(n);
            };
            // one run longer than kHistCap: record windows of kHistCap (each holds at most kHistCap of
            // its entries), each gathered in record order through the window's bitmap, then walked
            auto long_run = [&](uint32_t r, uint32_t c0) {
                const uint32_t e_lo = L.rp[r], len = L.rp[r + 1u] - e_lo;
                if (L.rn[r] >> 31) {  // a combined run is in record order: windows of kHistCap entries
                    for (uint32_t e = 0; e < len; e += kHistCap) {
                        const uint32_t m = min(kHistCap, len - e);
                        for (uint32_t i = tid; i < m; i += kHistThreads) L.skey2[i] = key_of(e_lo + e + i, r, c0);
                        __syncthreads();
                        walk(m);
                    }
                    return;
                }
                constexpr uint32_t kWinWords = kHistCap / 32u;
                for (uint32_t w0 = 0; w0 < kFlowChunk; w0 += kHistCap) {
                    for (uint32_t w = tid; w < kWinWords; w += kHistThreads) L.bm[w] = 0u;
                    __syncthreads();
                    for (uint32_t i = tid; i < len; i += kHistThreads) {
                        const uint32_t k = key_of(e_lo + i, r, c0), rec = k >> 13;
                        if (k != ~0u && rec >= w0 && rec < w0 + kHistCap)
                            atomicOr(&L.bm[(rec - w0) >> 5], 1u << ((rec - w0) & 31u));
                    }
                    __syncthreads();
                    const uint32_t n = bitmap_prefix(kWinWords);
                    if (n == 0u) continue;  // uniform
                    for (uint32_t i = tid; i < len; i += kHistThreads) {
                        const uint32_t k = key_of(e_lo + i, r, c0), rec = k >> 13;
                        if (k != ~0u && rec >= w0 && rec < w0 + kHistCap) L.skey2[rank_of(rec - w0)] = k;
                    }
                    __syncthreads();
                    walk(n);
                }
            };
            for (uint32_t c0 = cb0; c0 < cb1; c0 += kHistRuns) {
                const uint32_t nr = min(kHistRuns, cb1 - c0);
                if (c0 != cb0) {
                    vp = tid < nr ? col[c0 + tid] : 0u;
                    round(c0, nr);
                }
                // batches of whole runs up to kHistCap entries; a longer run alone, in record windows
                uint32_t r = 0;
                while (r < nr) {  // uniform: every thread walks the same runs
                    if (L.rp[r + 1u] - L.rp[r] > kHistCap) {
                        long_run(r, c0);
                        ++r;
                        continue;
                    }
                    // r1 = the largest run index with rp[r1] <= rp[r] + kHistCap (> r: run r fits)
                    uint32_t lo = r + 1u, hi = nr;
                    const uint32_t lim = L.rp[r] + kHistCap;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi + 1u) >> 1;
                        if (L.rp[mid] <= lim) lo = mid; else hi = mid - 1u;
                    }
                    batch(r, lo, L.rp[r], L.rp[lo], c0);
                    r = lo;
                }
                __syncthreads();
            }
        }
    };
    // pairs i: first the slow list's partitions (a workgroup each, every chunk; not in the counting
    // pass), then the split list's (partition, block) pairs numbered densely -- each split
    // partition takes the blocks it asked for (capped at nblk), so every workgroup gets some
    const uint32_t n_slow = (!COUNT && slow) ? slow[0] : 0u;
    uint32_t n = 0u, total = 0u;
    if (hot) {  // (uniform)
        n = min(hot[0], kHistListCap);
        static_assert(kHistListCap <= kHistThreads, "one listed partition per thread");
        const uint32_t nbt = tid < n ? min(max(hot[1u + tid] >> 16, 2u), nblk) : 0u;
        const uint32_t ex = block_scan(nbt, total);
        if (tid <= n) L.pairs[tid] = ex;  // (pairs[n] = total)
        __syncthreads();
    }
    for (uint32_t i = blockIdx.x; i < n_slow + total; i += gridDim.x) {  // (blocks of one partition adjacent)
        if (i < n_slow) {
            partition(slow[1u + i], 0u, 0u, 1u);
        } else {
            const uint32_t j = i - n_slow;
            uint32_t lo = 0u, hi = n - 1u;  // the split partition holding pair j
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1u) >> 1;
                if (L.pairs[mid] <= j) lo = mid; else hi = mid - 1u;
            }
            partition(hot[1u + lo] & 0xFFFFu, lo, j - L.pairs[lo], L.pairs[lo + 1u] - L.pairs[lo]);
        }
        __syncthreads();  // the LDS is re-initialised for the next partition
    }
}

// The split partitions' per-block slot counts -> their exclusive prefix over the blocks, in place
// (block b of a split partition starts slot s after blocks 0 .. b - 1).  Workgroup (partition, 32
// slots): thread (g, s) takes blocks 8 g .. 8 g + 7 of its slot, all loads in flight, then adds the
// earlier groups' sums.
constexpr uint32_t kHbSlots = 32, kHbPer = 8;
static_assert(kHbPer * (kHistThreads / kHbSlots) >= kHistMaxBlocks, "every block in a group");
__global__ __launch_bounds__(kHistThreads) void k_hist_blocks(const uint32_t* list, uint32_t* cnt, uint32_t nblk) {
    __shared__ uint32_t gsum[kHistThreads / kHbSlots][kHbSlots];
    const uint32_t li = blockIdx.x / (kFlowSlots / kHbSlots);
    if (li >= min(list[0], kHistListCap)) return;
    const uint32_t nb = min(max(list[1u + li] >> 16, 2u), nblk);  // (k_hist_general's blocks)
    const uint32_t g = threadIdx.x / kHbSlots, sl = (blockIdx.x % (kFlowSlots / kHbSlots)) * kHbSlots + threadIdx.x % kHbSlots;
    uint32_t* c = cnt + (size_t)li * nblk * kFlowSlots + sl;
    uint32_t x[kHbPer], run = 0u;
#pragma unroll
    for (uint32_t u = 0; u < kHbPer; ++u) {
        const uint32_t b = g * kHbPer + u;
        x[u] = b < nb ? c[(size_t)b * kFlowSlots] : 0u;
        run += x[u];
    }
    gsum[g][threadIdx.x % kHbSlots] = run;
    __syncthreads();
    run = 0u;
    for (uint32_t k = 0; k < g; ++k) run += gsum[k][threadIdx.x % kHbSlots];
#pragma unroll
    for (uint32_t u = 0; u < kHbPer; ++u) {
        const uint32_t b = g * kHbPer + u;
        if (b < nb) c[(size_t)b * kFlowSlots] = run;
        run += x[u];
    }
}

uint64_t flow_history_cnt_bytes(uint32_t chunks) {  // the split list (count + entries), then the counts
    const uint32_t nblk = std::min<uint32_t>(kHistMaxBlocks, (chunks + kHistBlockChunks - 1u) / kHistBlockChunks);
    return nblk > 1u ? (kHistListCap + 1u) * 4ull + (uint64_t)kHistListCap * nblk * kFlowSlots * 4u : 0u;
}
hipError_t launch_flow_history(const FlowParams& p, uint32_t chunks, uint32_t* hist_slot, uint8_t* hist,
                               uint32_t* n_hist, uint32_t* slow, uint32_t* cnt, hipStream_t s) {
    if (chunks == 0u) chunks = 1u;
    const uint32_t nblk =
        cnt ? std::min<uint32_t>(kHistMaxBlocks, (chunks + kHistBlockChunks - 1u) / kHistBlockChunks) : 1u;
    uint32_t* hot = nblk > 1u ? cnt : nullptr;  // the split list; its counts after it
    uint32_t* hcnt = hot ? hot + kHistListCap + 1u : nullptr;
    hipLaunchKernelGGL(k_hist_scan, dim3(1), dim3(1024), 0, s, p.partials, p.parts, p.part_base, n_hist, slow, hot);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hist_uniform, dim3(p.parts), dim3(kHistThreads), 0, s, p, chunks, hist_slot, hist, slow, hot);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (!hot) {  // the listed partitions (a handful unless the batch is skewed): a grid-stride loop
        hipLaunchKernelGGL(k_hist_general<false>, dim3(min(p.parts, 512u)), dim3(kHistThreads), 0, s, p, chunks,
                           hist_slot, hist, slow, nullptr, nullptr, 1u);
        return hipGetLastError();
    }
    // the split ones' per-block slot counts, their prefix over the blocks, then the slow list's
    // partitions and the split ones' blocks in one launch
    hipLaunchKernelGGL(k_hist_general<true>, dim3(kHistSplitGrid), dim3(kHistThreads), 0, s, p, chunks, hist_slot, hist,
                       nullptr, hot, hcnt, nblk);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hist_blocks, dim3(kHistListCap * (kFlowSlots / kHbSlots)), dim3(kHistThreads), 0, s, hot, hcnt,
                       nblk);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hist_general<false>, dim3(kHistSplitGrid), dim3(kHistThreads), 0, s, p, chunks, hist_slot,
                       hist, slow, hot, hcnt, nblk);
    return hipGetLastError();
}

}  // namespace fbk
