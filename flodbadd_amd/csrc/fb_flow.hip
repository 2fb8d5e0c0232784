// fb_flow.hip -- gfx950 session (flow) table: upsert of SESSION records + integer counters.
//
// Replaces the per-packet DashMap upsert of process_parsed_packet (src/packets.rs:329-535):
// Entry::Occupied -> update_session_stats counters (src/packets.rs:111-120), Entry::Vacant ->
// new SessionInfo with the first packet's counters (src/packets.rs:383-391), and the
// PACKET_STATS new/updated counters (src/packets.rs:334-347).
//
// Design (owner-computes, no global atomics on the data path).  A per-packet global atomic
// design is bound by the memory-side atomic rate: 3 counter adds per packet ran at ~17 G
// atomics/s = 1.73 ms per 10M-record batch on MI355X (profiles/r01_c4_kernel_stats.csv).
// Instead the table is split into P partitions of kFlowSlots slots (fb_internal.h) and a batch
// is applied in three launches:
//   K1 k_flow_bucket    one workgroup per chunk of kFlowChunk record slots: LDS histogram of the
//                       records' partitions (handed over by the fused parse, else hashed here),
//                       exclusive scan, then a counting-sort scatter of each record's SLOT INDEX
//                       (4 B) into the chunk's region of `entries` (partition-major inside the
//                       chunk); row b of `rows` = (start, count) per partition.
//   K1c k_flow_combine  the hot (chunk, partition) groups K1 listed are reduced per key (skewed
//                       popularity: one hot flow would otherwise run through one CU); a key met
//                       more than once becomes one combined entry in `comb`, its index word
//                       kIdxCombined | id.
//   K1t k_flow_transpose rows[chunk][part] -> cols[part][chunk] (so K2 reads its column
//                       contiguously), and each partition's entries summed: the partitions past
//                       twice the mean are listed for K2's leading workgroups.
//   K2 k_flow_apply     one workgroup per partition (the listed ones first, then the rest in
//                       order: under Zipf(1.1) a partition holding a flow K1c leaves plain takes
//                       up to ~210 us, and in partition order such workgroups started up to
//                       ~280 us into the launch -- K2 405 -> 330 us, tools/experiments/
//                       flow_trace.py, profiles/r05_k2_experiments.txt): loads the partition's slot heads into LDS,
//                       gathers its entries' records (or combined entries) from every chunk,
//                       finds/inserts each key in the slice, adds the counters and reduces the
//                       ordered state with LDS atomics, folds the ordered state once per slot,
//                       writes the slice back.
// K1 writing 4-B indices instead of 64-B entries (records gathered by K2 itself) cut K1 from 437
// to 140 us per C4 batch; K2 gathers 56-B records instead of 64-B entries and pipelines them.
// Counters are integer sums, so results are bit-exact whatever the order (the order-dependent
// history state is reduced to min/max/or, see K2); new_sessions counts
// the keys inserted (each key is inserted once), updated_sessions the remaining records.
// The reference hashes Session with SipHash under a random per-process key (dashmap 6.1.0
// RandomState), so no hash value is a parity target; this table uses fb_flow_hash (below), a
// deterministic 64-bit mix of the 40-B session_key, identical on host and device.
#include "fb_internal.h"

namespace fbk {

// flow_hash_words / part_of: fb_internal.h (the parse kernel computes the partition too).

#ifdef FB_FLOW_TRACE
// -DFB_FLOW_TRACE (never the product): per K2 workgroup (partition, up to kFlowTrParts) the
// real-time ticks of its start, the end of its entry loop and its end, its entries (low word) and
// its busiest slot's history characters (high word); per K1c workgroup its start, its end, its
// groups, its records and the ticks its groups spent in each phase (group fetch, table init,
// reduce, numbering, order bitmap, pack, combined entries) (tools/experiments/flow_trace.py,
// fb_flow_trace_last)
constexpr uint32_t kFlowTrParts = 8192u;
constexpr uint32_t kK1cTrWords = 12u;  // start, end, groups, records, 7 phase totals, 0
__device__ unsigned long long g_k2_trace[kFlowTrParts * 4u];
__device__ unsigned long long g_k1c_trace[1024u * kK1cTrWords];
__device__ __forceinline__ unsigned long long flow_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define FLOWTR(stmt) do { stmt; } while (0)
#else
#define FLOWTR(stmt) do { } while (0)
#endif

// Inclusive wave scan + block exclusive scan of one u32 per thread (blockDim multiple of 64).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63u) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0u, tot = 0u;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint32_t s = wsum[w];
        before += w < wave ? s : 0u;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0u) sh[wave] = v;
    __syncthreads();
    unsigned long long t = 0ull;
    for (uint32_t w = 0; w < blockDim.x / 64u; ++w) t += sh[w];
    __syncthreads();
    return t;
}

// A (chunk, partition) group of at least this many records (and 4x the chunk's mean) is combined
// per key by k_flow_combine before K2.
#ifndef FB_COMB_MIN
#define FB_COMB_MIN 64  // (48 until K2 started its heavy partitions first; with that order, C4 Zipf(1.1)
                        // pipelined 10,706 -> 10,924 and one stream 10,105 -> 10,317 at 64, while 96 /
                        // 128 gained pipelined and lost one stream -- a partition whose flow stays plain
                        // then takes ~390 us in K2; profiles/r05_k2_experiments.txt)
#endif
constexpr uint32_t kCombMin = FB_COMB_MIN;

// pkt_index of a combined group's first / last record `rec` (with entries rec IS the pkt_index)
__device__ __forceinline__ uint32_t rec_pkt(const FlowParams& P, uint32_t rec) {
    if (P.ent) return rec;
    return reinterpret_cast<const uint32_t*>(P.recs + rec)[13];
}

// FB_HIST_CHARS bit of a map_tcp_flags character (16 = not a history character), branch-free (a
// switch here compiled to a divergent compare tree of ~100 scalar mask instructions per entry):
// c & 31 tells the classes apart (S H F R A and > < -), c >= 96 marks the responder's lower-case
// letter (bit + 1), and the result is checked against the table "SsHhFfRr><Aa-".
constexpr unsigned long long hist_nibbles(uint32_t half) {
    const char cs[8] = {'S', 'H', 'F', 'R', '>', '<', 'A', '-'};
    const uint32_t bs[8] = {0u, 2u, 4u, 6u, 8u, 9u, 10u, 12u};
    unsigned long long v = ~0ull;
    for (int j = 0; j < 8; ++j) {
        const uint32_t k = (uint32_t)cs[j] & 31u;
        if ((k >> 4) == half) v = (v & ~(15ull << (4u * (k & 15u)))) | ((unsigned long long)bs[j] << (4u * (k & 15u)));
    }
    return v;
}
constexpr unsigned long long hist_chars(uint32_t half) {
    const char t[13] = {'S', 's', 'H', 'h', 'F', 'f', 'R', 'r', '>', '<', 'A', 'a', '-'};
    unsigned long long v = 0ull;
    for (uint32_t j = 8u * half; j < 8u * half + 8u && j < 13u; ++j) v |= (unsigned long long)(uint8_t)t[j] << (8u * (j & 7u));
    return v;
}
__device__ __forceinline__ uint32_t hist_bit(uint32_t c) {
    constexpr unsigned long long kN0 = hist_nibbles(0), kN1 = hist_nibbles(1), kC0 = hist_chars(0), kC1 = hist_chars(1);
    const uint32_t k = c & 31u;
    const uint32_t nib = (uint32_t)(((k < 16u ? kN0 : kN1) >> (4u * (k & 15u))) & 15u);
    const uint32_t b = nib + (c >= 96u ? 1u : 0u);
    const uint32_t want = (uint32_t)(((b < 8u ? kC0 : kC1) >> (8u * (b & 7u))) & 0xFFu);
    return (nib != 15u && b < 13u && want == c) ? b : 16u;
}

// The entry word's history code of a record: 0 without history character (not TCP), else 1 + the
// FB_HIST_CHARS index of its map_tcp_flags character (hist_char | tcp_flags << 8 | has_flags << 16
// as in FlowEntry word 14, or the fused parse's partition word: char << 16 | has_flags << 24).
__device__ __forceinline__ uint32_t hist_code(uint32_t has_flags, uint32_t ch) {
    const uint32_t b = hist_bit(ch);
    return has_flags && b < 13u ? b + 1u : 0u;
}

// K1's LDS histogram / cursors: one u32 per partition, or (more than kFlowPackedParts partitions)
// two u16 halves per word -- a chunk holds < 2^16 records, so no half carries into the other.
struct PartHist {
    uint32_t* w;
    bool packed;
    __device__ __forceinline__ uint32_t add(uint32_t p) const {  // returns the old count / cursor
        if (!packed) return atomicAdd(&w[p], 1u);
        const uint32_t sh = 16u * (p & 1u);
        return (atomicAdd(&w[p >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
    __device__ __forceinline__ uint32_t get(uint32_t p) const {
        return packed ? reinterpret_cast<const uint16_t*>(w)[p] : w[p];
    }
    __device__ __forceinline__ void set(uint32_t p, uint32_t v) const {
        if (packed) reinterpret_cast<uint16_t*>(w)[p] = (uint16_t)v;
        else w[p] = v;
    }
};
__host__ __device__ inline uint32_t part_hist_bytes(uint32_t parts) {
    return parts > kFlowPackedParts ? parts * 2u : parts * 4u;
}
// K1 stages its scatter in LDS (the chunk's 4-B words) when the histogram leaves room for it
__host__ __device__ inline bool k1_staged(uint32_t parts) { return parts <= kFlowPackedParts; }
__host__ __device__ inline uint32_t k1_lds_bytes(uint32_t parts) {
    return part_hist_bytes(parts) + (k1_staged(parts) ? kFlowChunk * 4u : 0u);
}
static_assert(kFlowChunk < 65536u, "packed K1 counters hold a chunk's records");

// ---------------------------------------------------------------------------------------------
// K1: bucket one chunk of records by partition (counting sort in LDS).
__global__ __launch_bounds__(kFlowK1Threads) void k_flow_bucket(const FlowParams P) {
    extern __shared__ uint32_t hist_w[];  // part_hist_bytes(P.parts)
    const PartHist hist{hist_w, P.parts > kFlowPackedParts};
    __shared__ uint32_t wsum[kFlowK1Threads / 64];
    const uint32_t n = batch_records(P);
    if (blockIdx.x == 0 && threadIdx.x == 0 && !P.seg && P.stats->n_session > (unsigned long long)P.max_recs)
        atomicOr(P.error, 8u);  // more records than the update scratch holds: the rest is dropped
    if (P.order)  // K2's partition order of this update (K1t sums into it)
        for (uint32_t j = blockIdx.x * kFlowK1Threads + threadIdx.x; j < P.parts + kK2Lead + 1u;
             j += gridDim.x * kFlowK1Threads)
            P.order[j] = 0u;
    const uint32_t base = blockIdx.x * kFlowChunk;
    if (base >= n) return;
    const uint32_t cnt = min(kFlowChunk, n - base);
    const fb_pkt_out* R = P.recs + base;
    for (uint32_t j = threadIdx.x; j < part_hist_bytes(P.parts) / 4u; j += kFlowK1Threads) hist_w[j] = 0u;
    // every thread owns the chunk's slots threadIdx.x + j * kFlowK1Threads; their partitions stay in
    // registers from the histogram pass to the scatter pass, and each pass issues all its loads
    // before the first LDS atomic (a loop of load -> atomic iterations waits a full memory round
    // trip per record)
    constexpr uint32_t kPer = kFlowChunk / kFlowK1Threads;
    static_assert(kFlowChunk % kFlowK1Threads == 0, "whole records per thread");
    uint32_t pv[kPer];  // partition of each owned slot, ~0u: no record
    if (P.rec_part) {   // partitions from the parse of this batch (fb_process_seg_dev): 4 B per record
        // every slot's segment count word (one per wave: 64 consecutive slots) and partition word
        // loaded unconditionally, then masked: a load that waited on the validity test would put
        // two dependent round trips per slot in sequence (K1 142 -> DESIGN)
        // (the null test of P.seg outside the loops: inside, the compiler waited for each load
        // at the join of its branch)
        uint32_t sw[kPer];
        if (P.seg) {
#pragma unroll
            for (uint32_t j = 0; j < kPer; ++j) {
                const uint32_t k = min(threadIdx.x + j * kFlowK1Threads, cnt - 1u);
                sw[j] = P.seg[(base + k) >> 6];
                pv[j] = P.rec_part[base + k];
            }
        } else {
#pragma unroll
            for (uint32_t j = 0; j < kPer; ++j) {
                const uint32_t k = min(threadIdx.x + j * kFlowK1Threads, cnt - 1u);
                sw[j] = 0xFFFFu;
                pv[j] = P.rec_part[base + k];
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t k = threadIdx.x + j * kFlowK1Threads;
            // the parse's word: partition | unit offset << 16 | IPv6 << 23 (kRec*, fb_internal.h)
            if (!(k < cnt && ((base + k) & 63u) < (sw[j] & 0xFFFFu))) pv[j] = ~0u;
        }
    } else {            // hashed here, four records' key loads in flight at a time
        constexpr uint32_t kG = 4;
#pragma unroll
        for (uint32_t j0 = 0; j0 < kPer; j0 += kG) {
            uint4 a[kG], b[kG];
            uint2 c[kG];
            uint32_t m[kG];
            bool ok[kG];
#pragma unroll
            for (uint32_t u = 0; u < kG; ++u) {
                const uint32_t k = threadIdx.x + (j0 + u) * kFlowK1Threads;
                ok[u] = k < cnt && slot_valid(P, base + k);
                const uint32_t* r = reinterpret_cast<const uint32_t*>(R + (ok[u] ? k : 0u));
                a[u] = ld_u4(r);
                b[u] = ld_u4(r + 4);
                c[u] = ld_u2(r + 8);
                m[u] = r[12];  // flags | meta << 8 | hist_char << 16
            }
#pragma unroll
            for (uint32_t u = 0; u < kG; ++u) {
                const uint32_t key[10] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w, c[u].x,
                                          c[u].y & 0xFFFFu};
                const uint32_t code = hist_code((m[u] >> 8) & FB_META_HAS_FLAGS, (m[u] >> 16) & 0xFFu);
                pv[j0 + u] = ok[u] ? part_of(flow_hash_words(key), P.part_shift) | code << 16 : ~0u;
            }
        }
    }
    __syncthreads();  // hist zeroed
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j)
        if (pv[j] != ~0u) hist.add(pv[j] & kRecPartMask);
    __syncthreads();
    // exclusive scan of hist[0..parts): each thread owns E consecutive partitions
    const uint32_t E = (P.parts + kFlowK1Threads - 1u) / kFlowK1Threads;
    const uint32_t j0 = threadIdx.x * E;
    uint32_t local = 0u;
    for (uint32_t j = j0; j < j0 + E && j < P.parts; ++j) local += hist.get(j);
    uint32_t total;
    uint32_t run = block_excl_scan(local, wsum, total);
    uint32_t* row = P.rows + (size_t)blockIdx.x * P.parts;
    const uint32_t hot_min = max(kCombMin, 4u * ((cnt + P.parts - 1u) / P.parts));
    static_assert(kFlowMaxParts / kFlowK1Threads <= 64u, "a thread's partitions fit the hot mask");
    unsigned long long hot = 0ull;  // this thread's hot groups (bit j - j0), handed to k_flow_combine
    uint32_t n_hot = 0u;
    for (uint32_t j = j0; j < j0 + E && j < P.parts; ++j) {
        const uint32_t c = hist.get(j);
        row[j] = run | (c << 16);  // run < kFlowChunk <= 2^15: bit 15 is k_flow_combine's mark
        if (c >= hot_min) {
            hot |= 1ull << (j - j0);
            ++n_hot;
        }
        hist.set(j, run);  // becomes the scatter cursor
        run += c;
    }
    if (P.hot) {  // one list slot atomic per workgroup (one per group serialised ~19K same-address
                  // atomics per Zipf C4 batch: K1 223 -> DESIGN us)
        __shared__ uint32_t s_hot0;
        uint32_t tot_hot;
        uint32_t h = block_excl_scan(n_hot, wsum, tot_hot);
        if (tot_hot != 0u) {
            if (threadIdx.x == 0) s_hot0 = atomicAdd(P.ctl, tot_hot);
            __syncthreads();
            h += s_hot0;
            for (; hot; hot &= hot - 1ull, ++h)
                if (h < P.hot_cap) P.hot[h] = blockIdx.x << 16 | (j0 + (uint32_t)__builtin_ctzll(hot));
        }
    }
    __syncthreads();
    // scatter: entry position -> the record's slot index | its history code, or (entries from the
    // fused parse) its update entry's unit index | IPv6 << 28 (4 B); K2 gathers the record / entry
    // Up to kFlowPackedParts partitions the words are scattered into an LDS copy of the chunk's
    // region and stored coalesced: scattered 4-B global stores left L2 partial lines that were
    // written back piecemeal (C4: 267 MB written per batch for 42 MB of words).
    uint32_t* out = P.entries + base;
    const bool staged = k1_staged(P.parts);
    uint32_t* stg = hist_w + part_hist_bytes(P.parts) / 4u;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        if (pv[j] == ~0u) continue;
        const uint32_t k = threadIdx.x + j * kFlowK1Threads;
        const uint32_t d = hist.add(pv[j] & kRecPartMask);
        const uint32_t w = P.rec_part ? ((base + k) >> 6) * kUpdUnitsPerSeg + ((pv[j] >> kRecUnitShift) & 127u) |
                                            ((pv[j] & kRecV6) ? kEntV6 : 0u)
                                      : (base + k) | (pv[j] >> 16) << kEntCodeShift;
        if (staged) stg[d] = w;
        else out[d] = w;
    }
    if (staged) {
        __syncthreads();
        uint4* o4 = reinterpret_cast<uint4*>(out);  // (base is a multiple of kFlowChunk: 16-B aligned)
        const uint4* s4 = reinterpret_cast<const uint4*>(stg);
        for (uint32_t q = threadIdx.x; q < total / 4u; q += kFlowK1Threads) o4[q] = s4[q];
        if (threadIdx.x < (total & 3u)) out[(total & ~3u) + threadIdx.x] = stg[(total & ~3u) + threadIdx.x];
    }
}

// ---------------------------------------------------------------------------------------------
// K1t: rows[chunk][part] -> cols[part][chunk_stride]
__global__ __launch_bounds__(256) void k_flow_transpose(const FlowParams P, uint32_t chunks) {
    __shared__ uint32_t tile[64][65];
    const uint32_t p0 = blockIdx.x * 64u, c0 = blockIdx.y * 64u;
    const uint32_t tx = threadIdx.x & 63u, ty = threadIdx.x >> 6;
    if (P.ctl && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {  // k_flow_combine is done with them
        P.ctl[0] = 0u;
        P.ctl[1] = 0u;
        P.ctl[2] = 0u;
        P.ctl[3] = 0u;
    }
    for (uint32_t y = ty; y < 64u; y += 4u) {
        const uint32_t c = c0 + y, p = p0 + tx;
        tile[y][tx] = (c < chunks && p < P.parts) ? P.rows[(size_t)c * P.parts + p] : 0u;
    }
    __syncthreads();
    // each partition's entries (a wave holds one partition's 64 chunks of the tile) summed into
    // P.order; the partition whose sum passes twice the mean joins K2's leading partitions.  Only a
    // tile holding at least its share of that (the tiles of a heavy partition do) adds with a
    // returned value -- the others' adds are fire-and-forget, so a uniform batch waits on none
    const uint32_t lead_min = max(64u, 2u * (uint32_t)(((unsigned long long)chunks * kFlowChunk) / P.parts));
    const uint32_t tile_min = lead_min / ((chunks + 63u) / 64u);
    for (uint32_t y = ty; y < 64u; y += 4u) {
        const uint32_t p = p0 + y, c = c0 + tx;
        const uint32_t w = tile[tx][y];
        if (p < P.parts && c < chunks) P.cols[(size_t)p * P.chunk_stride + c] = w;
        if (P.order && p < P.parts) {  // (uniform per wave)
            uint32_t sum = c < chunks ? w >> 16 : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
            if (tx == 0u && sum != 0u && sum < tile_min) {
                __hip_atomic_fetch_add(P.order + p, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (tx == 0u && sum != 0u) {
                const uint32_t old = atomicAdd(P.order + p, sum);
                if (old < lead_min && old + sum >= lead_min) {
                    const uint32_t i = atomicAdd(P.order + P.parts + kK2Lead, 1u);
                    if (i < kK2Lead) {
                        P.order[P.parts + i] = p;
                        atomicOr(P.order + p, 1u << 31);
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K2: apply one partition's entries to its LDS-resident slice.
//
// LDS: the slots' first 96 B (tag, key, counters) + a 40-B per-slot batch scratch = 68 KiB, so two
// workgroups share a CU and one's slice load / write-back overlaps the other's apply (at one
// workgroup per CU, with the ordered fields in LDS too, the phases ran back to back).
//
// Ordered state (src/packets.rs:187-198, 410-426).  Entries reach K2 in no particular order, so
// everything order-dependent is reduced to order-independent LDS atomics over the record slot
// `rec` (batch order) in the scratch, then folded into the slot's ordered fields (in HBM, read
// and written once per touched slot) at the end:
//   first / last packet  = min / max rec; end (first FIN/RST) = min rec of the TCP records with
//                          FIN or RST; their pkt_index (and the end packet's character) are read
//                          back from the records
//   history              = count, OR of the FB_HIST_CHARS bits, first rec of S s H h.
// conn_state at the end packet is determine_conn_state over the characters the history holds
// then: the flow's mask from earlier batches | S s H h whose first occurrence is at or before the
// end record | the end packet's own character.  F f R r need no first occurrence: each comes from
// a FIN or RST packet, and the first of those IS the end packet (the reference's string tests
// `history.contains(c)` only ask which characters are present).
constexpr uint32_t kSlotWords = 12;  // u64 words of a slot kept in LDS: tag, key[5], counters[6]
constexpr uint32_t kScrU32 = 12;     // per-slot batch scratch, u32 words (8-B aligned: three u64 keys)
#ifndef FB_K2_TAGS
#define FB_K2_TAGS 1
#endif
constexpr uint32_t kK2Lds = kFlowSlots * (kSlotWords * 8 + kScrU32 * 4 + (FB_K2_TAGS ? 4 : 0));
constexpr uint32_t kTcpFinRst = 0x01u | 0x04u;
#ifndef FB_K2_CPT
#define FB_K2_CPT 1
#endif
constexpr uint32_t kK2Cpt = FB_K2_CPT;
// (kK2Cpt: bucketing chunks per K2 thread and round; C4: 512 chunks, one round)
// scratch words: first / last packet as u64 keys rec << 32 | pkt_index (min / max), the end packet
// as rec << 37 | its FB_HIST_CHARS bit << 32 | pkt_index (min) -- so the fold needs no record
// read-back --, the mask, the history count, the first rec of S s H h
constexpr uint32_t kScFirst = 0, kScLast = 2, kScEnd = 4, kScMask = 6, kScCount = 7, kScChar = 8;  // kScChar..+3
constexpr uint32_t kScOrd = 4;  // after the fold: the slot's new ordered fields (2 uint4, 16-B aligned)
__device__ __forceinline__ unsigned long long* sc64(uint32_t* q, uint32_t w) {
    return reinterpret_cast<unsigned long long*>(q + w);
}
__device__ __forceinline__ unsigned long long end_key(uint32_t rec, uint32_t bit, uint32_t pkt) {
    return (unsigned long long)rec << 37 | (unsigned long long)bit << 32 | pkt;
}

__device__ __forceinline__ unsigned long long lds_ld(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// determine_conn_state: conn_state_of (fb_internal.h).

// Find or insert `key` in an LDS open-addressing table of kSlots slots of kStride u64 words
// (tag: 0 empty, 1 being inserted, hash | 2; then the 5 key words), home slot h32 & (kSlots-1).
// h32 = the low word of the key's hash, handed over by K1: home slot and a 32-bit tag filter
// (the 64-bit tag is only computed to insert).  Returns 1 inserted, 0 found (*slot set),
// -1 table full, -2 spin expired.
template <uint32_t kStride, uint32_t kSlots>
__device__ __forceinline__ int lds_upsert(unsigned long long* tab, const uint32_t key[10], uint32_t h32,
                                          uint32_t& slot) {
    const uint32_t want32 = h32 | 2u;
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    uint32_t i = h32 & (kSlots - 1u);
    int result = -1;
    for (uint32_t probe = 0; probe < kSlots; ++probe) {
        unsigned long long* s = tab + (size_t)i * kStride;
        unsigned long long t = lds_ld(s);
        if (t == 0ull) {
            const unsigned long long old = atomicCAS(s, 0ull, 1ull);
            if (old == 0ull) {
                s[1] = kw0;
                s[2] = kw1;
                s[3] = kw2;
                s[4] = kw3;
                s[5] = kw4;
                __hip_atomic_store(s, (unsigned long long)want32, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                result = 1;
                break;
            }
            t = old;
        }
        uint32_t spins = 0u;
        while (t == 1ull) {  // another lane of this workgroup is publishing the slot's key
            __builtin_amdgcn_s_sleep(1);
            t = lds_ld(s);
            if (++spins > (1u << 22)) return -2;
        }
        if ((uint32_t)t == want32 && s[1] == kw0 && s[2] == kw1 && s[3] == kw2 && s[4] == kw3 && s[5] == kw4) {
            result = 0;
            break;
        }
        i = (i + 1u) & (kSlots - 1u);
    }
    slot = i;
    return result;
}

// Lookup only (no concurrent inserts): the slot of `key`, or ~0u.
template <uint32_t kStride, uint32_t kSlots>
__device__ __forceinline__ uint32_t lds_find(const unsigned long long* tab, const uint32_t key[10], uint32_t h32) {
    const uint32_t want32 = h32 | 2u;
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    uint32_t i = h32 & (kSlots - 1u);
    for (uint32_t probe = 0; probe < kSlots; ++probe) {
        const unsigned long long* s = tab + (size_t)i * kStride;
        const unsigned long long t = s[0];
        if (t == 0ull) return ~0u;
        if ((uint32_t)t == want32 && s[1] == kw0 && s[2] == kw1 && s[3] == kw2 && s[4] == kw3 && s[5] == kw4)
            return i;
        i = (i + 1u) & (kSlots - 1u);
    }
    return ~0u;
}

// Lookup while other lanes may be inserting (tags read with acquire, so a published tag's key
// words are visible); a slot being inserted (tag 1) is probed past.  ~0u: not (yet) present --
// the caller then takes lds_upsert, which waits on such a slot.  Steady-state batches mostly
// update existing flows, so this branch-light loop is the common path and the upsert with its
// claim / spin states the rare one (it costs ~40 scalar mask instructions per probe even when
// nothing spins).
template <uint32_t kStride, uint32_t kSlots>
__device__ __forceinline__ uint32_t lds_lookup(unsigned long long* tab, const uint32_t key[10], uint32_t h32) {
    const uint32_t want32 = h32 | 2u;
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    uint32_t i = h32 & (kSlots - 1u);
    for (uint32_t probe = 0; probe < kSlots; ++probe) {
        unsigned long long* s = tab + (size_t)i * kStride;
        // the tag, then the key words, issued together (one wait): a wave's LDS reads are served
        // in order and a publisher writes the key before its release store of the tag, so a
        // published tag read first implies its key words; the compare is branch-free
        const unsigned long long t = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
        const unsigned long long a = s[1], b = s[2], c = s[3], d = s[4], e = s[5];
        if (t == 0ull) break;
        if (((uint32_t)t == want32) & (a == kw0) & (b == kw1) & (c == kw2) & (d == kw3) & (e == kw4)) return i;
        i = (i + 1u) & (kSlots - 1u);
    }
    return ~0u;
}

// K2's probe over a tag array: tags[i] = the low word of slot i's tag (0 empty, 1 being inserted,
// h32 | 2), kept beside the slot heads.  A lookup reads the 8 tags of the probe's 32-B group with
// two LDS reads, compares them in registers, and reads a slot's key words only on a tag match; it
// stops at the group's first empty slot.  At the steady-state load (C4: 1.45M flows in 2^21
// slots, 0.69) a linear probe's length has a long tail and a wave runs its loop as often as its
// longest lane needs: 8 slots per step cut that from ~a dozen steps of six 8-B slot reads to
// one or two group reads.
__device__ __forceinline__ uint32_t k2_lookup(const uint32_t* tags, const unsigned long long* tab,
                                              const uint32_t key[10], uint32_t h32) {
    const uint32_t want = h32 | 2u;
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    const uint32_t start = h32 & (kFlowSlots - 1u);
    uint32_t grp = start >> 3, live = 0xFFu & (0xFFu << (start & 7u));  // group positions at or past the home slot
    for (uint32_t n = 0; n < kFlowSlots / 8u; ++n) {
        // (re)read every step: other lanes publish tags; a wave's LDS reads are served in order and
        // a publisher writes the key words before its release store of the tag
        asm volatile("" ::: "memory");
        const uint4* tg = reinterpret_cast<const uint4*>(tags + grp * 8u);
        const uint4 a = tg[0], b = tg[1];
        asm volatile("" ::: "memory");
        const uint32_t t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t match = 0u, empty = 0u;
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) {
            match |= (t[j] == want ? 1u : 0u) << j;
            empty |= (t[j] == 0u ? 1u : 0u) << j;
        }
        empty &= live;
        match &= live & (empty ? (empty & (0u - empty)) - 1u : 0xFFu);  // before the first empty
        while (match) {
            const uint32_t i = grp * 8u + (uint32_t)__builtin_ctz(match);
            const unsigned long long* s = tab + (size_t)i * kSlotWords;
            if ((s[1] == kw0) & (s[2] == kw1) & (s[3] == kw2) & (s[4] == kw3) & (s[5] == kw4)) return i;
            match &= match - 1u;
        }
        if (empty) break;
        grp = (grp + 1u) & (kFlowSlots / 8u - 1u);
        live = 0xFFu;
    }
    return ~0u;  // absent, being inserted, or past a full table: the caller takes k2_upsert
}

// Find or insert through the tag array (claim: CAS of the slot's tag 0 -> 1, then the key words
// and the 64-bit slot tag, then the release store of h32 | 2).  Same results as lds_upsert.
__device__ __forceinline__ int k2_upsert(uint32_t* tags, unsigned long long* tab, const uint32_t key[10],
                                         uint32_t h32, uint32_t& slot) {
    const uint32_t want = h32 | 2u;
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    uint32_t i = h32 & (kFlowSlots - 1u);
    int result = -1;
    for (uint32_t probe = 0; probe < kFlowSlots; ++probe) {
        unsigned long long* s = tab + (size_t)i * kSlotWords;
        uint32_t t = __hip_atomic_load(tags + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (t == 0u) {
            const uint32_t old = atomicCAS(tags + i, 0u, 1u);
            if (old == 0u) {
                s[1] = kw0;
                s[2] = kw1;
                s[3] = kw2;
                s[4] = kw3;
                s[5] = kw4;
                s[0] = (unsigned long long)want;  // slot tag | segment_count 0 << 32
                __hip_atomic_store(tags + i, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                result = 1;
                break;
            }
            t = old;
        }
        uint32_t spins = 0u;
        while (t == 1u) {  // another lane of this workgroup is publishing the slot's key
            __builtin_amdgcn_s_sleep(1);
            t = __hip_atomic_load(tags + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (++spins > (1u << 22)) return -2;
        }
        if (t == want && s[1] == kw0 && s[2] == kw1 && s[3] == kw2 && s[4] == kw3 && s[5] == kw4) {
            result = 0;
            break;
        }
        i = (i + 1u) & (kFlowSlots - 1u);
    }
    slot = i;
    return result;
}

// K2's find-or-insert: lookup first (steady-state batches mostly update existing flows), then the
// claiming upsert.
__device__ __forceinline__ int k2_find_insert(unsigned long long* slice, uint32_t* tags, const uint32_t key[10],
                                              uint32_t h32, uint32_t& i) {
#if FB_K2_TAGS
    i = k2_lookup(tags, slice, key, h32);
    return i != ~0u ? 0 : k2_upsert(tags, slice, key, h32, i);
#else
    (void)tags;
    i = lds_lookup<kSlotWords, kFlowSlots>(slice, key, h32);
    return i != ~0u ? 0 : lds_upsert<kSlotWords, kFlowSlots>(slice, key, h32, i);
#endif
}

// Returns 1 if the key was inserted, 0 if it existed; -1 if the partition is full/spin expired.
__device__ __forceinline__ int apply_entry(unsigned long long* slice, uint32_t* tags, uint32_t* scr, const uint4 e0, const uint4 e1,
                                           const uint4 e2, const uint4 e3, uint32_t& slot, uint32_t* err) {
    const uint32_t orig = (e2.y >> 16) & 1u;
    const uint32_t key[10] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y & 0xFFFFu};
    uint32_t i;
    const int result = k2_find_insert(slice, tags, key, e3.w, i);
    if (result < 0) {
        atomicOr(err, result == -2 ? 16u : 4u);  // spin expired / partition full
        return -1;
    }
    unsigned long long* s = slice + (size_t)i * kSlotWords;
    // originator -> outbound_bytes/orig_pkts/orig_ip_bytes, else inbound/resp (packets.rs:111-120)
    atomicAdd(s + 6 + (orig ? 0 : 1), (unsigned long long)e2.z);
    atomicAdd(s + 8 + (orig ? 0 : 1), 1ull);
    atomicAdd(s + 10 + (orig ? 0 : 1), (unsigned long long)e2.w);
    slot = i;
    // ordered state into the batch scratch (see above)
    uint32_t* q = scr + (size_t)i * kScrU32;
    const uint32_t rec = e3.y;
    const unsigned long long pos = (unsigned long long)rec << 32 | e3.x;  // rec, pkt_index
    // a TCP packet with PSH ends a segment (src/packets.rs:140-160, 414-420): segment_count += 1 in
    // the slot head's high word, and the last packet's key carries the bit (in_segment = !PSH of the
    // flow's latest packet); pkt_index < 2^27 leaves bit 31 free
    const uint32_t psh = (e3.z & 0x10000u) && ((e3.z >> 8) & kTcpPsh) && (e2.y & 0xFFu) == 6u ? 1u : 0u;
    if (psh) atomicAdd(s, 1ull << 32);
    atomicMin(sc64(q, kScFirst), pos);
    atomicMax(sc64(q, kScLast), pos | (unsigned long long)psh << 31);
    // inserted by this batch: bit 16, and the session flags the reference stores at insert
    // (is_local_src/dst, is_self_src/dst of the canonical key, src/packets.rs:429-435) in bits 20-23
    // dst_service (src/packets.rs:441-466) in bit 15
    if (result == 1) atomicOr(q + kScMask, (1u << 16) | (e3.z & 0x00F00000u) | ((e3.z >> 24) & 1u) << 15);
    if (e3.z & 0x10000u) {                              // Some(flags): history.push(map_tcp_flags(..))
        atomicAdd(q + kScCount, 1u);
        const uint32_t b = hist_bit(e3.z & 0xFFu);
        if (b < 16u) atomicOr(q + kScMask, 1u << b);
        if (b < 4u) atomicMin(q + kScChar + b, rec);
        if ((e3.z >> 8) & kTcpFinRst) atomicMin(sc64(q, kScEnd), end_key(rec, b, e3.x));
    }
    return result;
}

// A combined entry (head e0..e3, tail t0..t3; layout in fb_internal.h): the same reductions with
// the group's partial sums / minima / maxima.  Its records' e_sort words point at agg_slot[id].
__device__ __forceinline__ int apply_combined(unsigned long long* slice, uint32_t* tags, uint32_t* scr,
                                              const FlowParams& P, const uint4 e0, const uint4 e1,
                                              const uint4 e2, const uint4 e3, const uint4 t0, const uint4 t1,
                                              const uint4 t2, const uint4 t3, uint32_t slot_base, uint32_t* agg_slot,
                                              uint32_t* err) {
    const uint32_t key[10] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y & 0xFFFFu};
    uint32_t i;
    const int result = k2_find_insert(slice, tags, key, e3.w, i);
    if (result < 0) {
        atomicOr(err, result == -2 ? 16u : 4u);
        if (agg_slot) agg_slot[e3.x] = ~0u;  // the history drops the group's characters (combined_slot)
        return -1;
    }
    unsigned long long* s = slice + (size_t)i * kSlotWords;
    const unsigned long long ob = t0.x | ((unsigned long long)t0.y << 32), ib = t0.z | ((unsigned long long)t0.w << 32);
    const unsigned long long oi = t1.x | ((unsigned long long)t1.y << 32), ri = t1.z | ((unsigned long long)t1.w << 32);
    const uint32_t op = t2.x & 0xFFFFu, rp = t2.x >> 16;
    if (op) {
        atomicAdd(s + 6, ob);
        atomicAdd(s + 8, (unsigned long long)op);
        atomicAdd(s + 10, oi);
    }
    if (rp) {
        atomicAdd(s + 7, ib);
        atomicAdd(s + 9, (unsigned long long)rp);
        atomicAdd(s + 11, ri);
    }
    if (agg_slot) agg_slot[e3.x] = slot_base + i;
    uint32_t* q = scr + (size_t)i * kScrU32;
    // the group's first / last / end records: their pkt_index (and the end's character) read here
    // -- combined entries are few
    atomicMin(sc64(q, kScFirst), (unsigned long long)e2.z << 32 | rec_pkt(P, e2.z));
    atomicMax(sc64(q, kScLast), (unsigned long long)e2.w << 32 | rec_pkt(P, e2.w) | (unsigned long long)((t3.w >> 15) & 1u) << 31);
    if (t3.w >> 16) atomicAdd(s, (unsigned long long)(t3.w >> 16) << 32);  // the group's PSH packets: segment_count
    const uint32_t hc = e3.z & 0xFFFFu;
    const uint32_t m = (e3.z >> 16) | (result == 1 ? (1u << 16) | ((t3.w & 0xFu) << 20) | ((t3.w >> 4) & 1u) << 15 : 0u);
    if (m) atomicOr(q + kScMask, m);
    if (hc) {
        atomicAdd(q + kScCount, hc);
        const uint32_t c[4] = {t2.z, t2.w, t3.x, t3.y};
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b)
            if (c[b] != ~0u) atomicMin(q + kScChar + b, c[b]);
        if (e3.y != ~0u) atomicMin(sc64(q, kScEnd), end_key(e3.y, (t3.w >> 8) & 31u, rec_pkt(P, e3.y)));
    }
    return result;
}

// Fold one slot's batch scratch into its ordered fields (after every entry was applied).  o0, o1 =
// the slot's ordered fields as loaded with the slice (first_seen, last_seen | end_seen, hist_len,
// hist_state); the first / last / end packets' pkt_index (and the end's character) are in the
// scratch keys.  The new ordered fields (bytes 96..127 of the slot) go to scratch words 4..11 --
// read before they are written -- so the write-back stores each touched slot as one whole line.
__device__ __forceinline__ void finish_slot(uint32_t* q, uint32_t batch, const uint4 o0, const uint4 o1, uint4* cc) {
    const unsigned long long first = *sc64(q, kScFirst);
    if (first == ~0ull) return;  // not touched by this batch
    const unsigned long long hi = (unsigned long long)batch << 32;
    const unsigned long long last = *sc64(q, kScLast), end = *sc64(q, kScEnd);
    const uint32_t flags = q[kScMask];
    const bool fresh = (flags & (1u << 16)) != 0u;  // new flow: start_time = its first packet, end_time None
    const unsigned long long first_seen = fresh ? hi | (uint32_t)first : (o0.x | (unsigned long long)o0.y << 32);
    unsigned long long end_seen = fresh ? FB_SEEN_NONE : (o1.x | (unsigned long long)o1.y << 32);
    // hist_state: hist_mask 0-12 | dst_service 15 | conn_state 16-19 | session flags 20-23 | end_mask 24-31
    const uint32_t state = fresh ? (flags & 0x00F00000u) : o1.w, len = fresh ? 0u : o1.z;
    const unsigned long long last_seen = hi | ((uint32_t)last & 0x7FFFFFFFu);
    // in_segment: the flow's latest packet was not a TCP PSH (bit 31 of the last key's low word)
    const uint32_t in_seg = ((uint32_t)last >> 31) ? 0u : kStateInSegment;
    const uint32_t mask = state & 0xFFFFu & ~kStateInSegment;
    // the update call of the first S, s, H, h of the flow (FB_CALL_NONE: none yet), kept beside the
    // table for the multi-GPU merge (it decides which of a rank's characters precede another rank's
    // end packet): written when a character first appears -- its mask bit was clear -- and whole at
    // insert, so nothing is read here
    if (cc) {
        uint32_t w[4];
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) w[b] = q[kScChar + b] != ~0u ? batch : FB_CALL_NONE;
        if (fresh) {
            *cc = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            uint32_t* c = reinterpret_cast<uint32_t*>(cc);
#pragma unroll
            for (uint32_t b = 0; b < 4u; ++b)
                if (w[b] != FB_CALL_NONE && !(mask & (1u << b))) c[b] = batch;
        }
    }
    uint32_t cs = state >> 16;
    if (end != ~0ull && end_seen == FB_SEEN_NONE) {  // the flow's first FIN/RST is in this batch
        const uint32_t end_rec = (uint32_t)(end >> 37);
        uint32_t m = mask | (1u << ((uint32_t)(end >> 32) & 31u));
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) m |= q[kScChar + b] <= end_rec ? 1u << b : 0u;
        cs = conn_state_of(m) | (cs & 0xF0u) | (m & 0xFFu) << 8;  // + the conn_state characters present at the end
        end_seen = hi | (uint32_t)end;
    }
    const uint4 t0 = make_uint4((uint32_t)first_seen, (uint32_t)(first_seen >> 32), (uint32_t)last_seen,
                                (uint32_t)(last_seen >> 32));
    const uint4 t1 = make_uint4((uint32_t)end_seen, (uint32_t)(end_seen >> 32), len + q[kScCount],
                                (mask | (flags & 0xFFFFu) | in_seg) | (cs << 16));
    uint4* t = reinterpret_cast<uint4*>(q + kScOrd);  // bytes 96..127 of the slot
    t[0] = t0;
    t[1] = t1;
}
static_assert(offsetof(FlowSlot, first_seen) == 96 && offsetof(FlowSlot, hist_state) == 124, "ordered fields at 96..127");

// ---------------------------------------------------------------------------------------------
// K1c: combine the records of one key inside the hot (chunk, partition) groups K1 listed.
//
// With skewed flow popularity one partition can hold a large share of a batch (Zipf(1.1): the
// hottest flow carries ~12 % of the records), and K2 gives a partition to ONE workgroup.  Here
// every hot group (>= kCombMin records and >= 4x the chunk's mean) is reduced per key in LDS by
// its own workgroup, spread over the whole chip, and rewritten in place: the records of keys met
// once stay as they are, packed to the front; each key met more than once becomes one combined
// entry (two units) behind them; the group's row count shrinks accordingly.  The partial sums are
// the same integer sums / minima / maxima K2 computes, so the result is bit-identical.
#ifndef FB_COMB_SLOTS
#define FB_COMB_SLOTS 256
#endif
#ifndef FB_COMB_GRID
#define FB_COMB_GRID 1024
#endif
// 256 keys (34 KiB of LDS, four workgroups per CU) x 1024 workgroups, groups >= 48 records: C4
// Zipf update 1.39 ms, against 1.74 ms at 512 keys x 512 / >= 24 (fixed cost per group: table
// init, barriers, the id atomic) and 1.50 ms at >= 48 with 512 keys (tools/sweep_flow.sh, ZIPF=1.1).
constexpr uint32_t kCombSlots = FB_COMB_SLOTS;  // keys past a full table stay plain entries
#ifndef FB_COMB_THREADS
#define FB_COMB_THREADS 256
#endif
constexpr uint32_t kCombThreads = FB_COMB_THREADS;
constexpr uint32_t kCombGrid = FB_COMB_GRID;
static_assert(kCombSlots % kCombThreads == 0, "each thread numbers kCombSlots / kCombThreads keys");
constexpr uint32_t kCfPk = 0, kCfFirst = 1, kCfLast = 2, kCfEnd = 3, kCfHcnt = 4, kCfMask = 5, kCfChar = 6,
                   kCfRecs = 10, kCfId = 11, kCfHash = 12, kCfMeta = 13, kCombF = 14;  // u32 fields of a key (kCfChar..+3)
// The reduce pass keeps each record's key slot (u8; 0xFF: none or slot 255) for the group's first
// kCombJc records, so the pack pass finds them without gathering the 56-B records again: K1c is
// bound by those random record reads (under Zipf(1.1) ~4.6M records per C4 batch sit in hot
// groups), not by its same-key LDS atomics (folding a hot key's lanes with wave reductions first
// measured slower: 318 -> 348-358 us).  C4 Zipf(1.1): K1c 371 -> 317 us.  (2560: the order bitmap
// below keeps the workgroup within 40 KiB; a Zipf(1.1) group holds up to ~2,460 records.)
#ifndef FB_COMB_JC
#define FB_COMB_JC 2560
#endif
constexpr uint32_t kCombJc = FB_COMB_JC;
#ifndef FB_COMB_U
#define FB_COMB_U 1  // (4: C4 Zipf K1c 328 -> 415 us)
#endif
constexpr uint32_t kCombU = FB_COMB_U;  // records per thread with their loads in flight together
// The group's records in record order for the history (e_sort): a bitmap of the records' places in
// the chunk (kFlowChunk bits) and its prefix popcounts; a record's rank = the set bits below it.
constexpr uint32_t kCombBm = kFlowChunk / 64u;
struct CombLds {
    unsigned long long tab[kCombSlots * 6];    // tag + key words (lds_upsert layout)
    unsigned long long bytes[kCombSlots * 4];  // outbound, inbound, orig ip, resp ip
    uint32_t f[kCombSlots * kCombF];
    unsigned long long bm[kCombBm];            // the group's records in the chunk
    uint16_t bmp[kCombBm];                     // exclusive prefix popcounts of bm
    uint8_t jc[kCombJc > 0 ? kCombJc : 1];     // the reduce pass's key slot per record
    uint32_t wsum[kCombThreads / 64];
    uint32_t base;
    uint32_t pool_next, pool_end;  // this workgroup's reserved combined-entry ids
    uint32_t grp_next;             // the group this workgroup took from the list
};
static_assert(sizeof(CombLds) <= 40u * 1024u, "four K1c workgroups per CU");
static_assert(kFlowChunk % 64u == 0u, "whole bitmap words");
constexpr uint32_t kCombBmPer = (kCombBm + kCombThreads - 1u) / kCombThreads;  // bitmap words per thread

__global__ __launch_bounds__(kCombThreads) void k_flow_combine(const FlowParams P) {
    __shared__ CombLds L;
    const uint32_t n_hot = min(P.ctl[0], P.hot_cap);
    // combined-entry ids: a workgroup reserves them `pool` at a time (one returned atomic per group on
    // one address serialised ~19K of them per Zipf C4 batch); the reservations leave most of comb_cap
    // (a quarter of the batch's records) to spare
    const uint32_t pool = max(1u, min(32u, P.comb_cap / (4u * gridDim.x)));
    if (threadIdx.x == 0) L.pool_next = L.pool_end = 0u;  // published by the group loop's first barrier
    uint32_t* E = P.entries;
    uint4* CE = reinterpret_cast<uint4*>(P.comb);
#ifdef FB_FLOW_TRACE
    const unsigned long long tr_t0 = flow_now();
    uint32_t tr_groups = 0u, tr_recs = 0u;
    unsigned long long tr_ph[7] = {}, tr_prev = tr_t0;
#define K1CPH(k) FLOWTR({ const unsigned long long t_ = flow_now(); tr_ph[k] += t_ - tr_prev; tr_prev = t_; })
#else
#define K1CPH(k) do { } while (0)
#endif
    // Groups are taken one at a time (ctl[3]), not by a fixed stride: their sizes vary by 50x under
    // skew (48 .. ~2,500 records), and with the stride the busiest workgroup held 2.2x the mean's
    // records (C4 Zipf(1.1) K1c 346 -> 288 us).  (Big groups first, from the back of the list:
    // K1c -5 us, K1 +7 us; not kept.)
    // The first group of a workgroup is its block index (a batch with few hot groups costs no
    // atomics in the workgroups that have none: 1,024 grabs on an empty list took 9 us).
    for (uint32_t it = 0;; ++it) {
        uint32_t h = blockIdx.x;
        if (it != 0u) {
            if (threadIdx.x == 0) L.grp_next = gridDim.x + atomicAdd(P.ctl + 3, 1u);
            __syncthreads();  // (every thread read the previous value before the last group's barriers)
            h = L.grp_next;
        }
        if (h >= n_hot) break;  // (uniform)
        const uint32_t grp = P.hot[h], chunk = grp >> 16, part = grp & 0xFFFFu;
        uint32_t* rowp = P.rows + (size_t)chunk * P.parts + part;
        const uint32_t row = *rowp, cnt = row >> 16;
        FLOWTR(++tr_groups; tr_recs += cnt);
        K1CPH(0);
        const size_t s0 = (size_t)chunk * kFlowChunk + (row & 0xFFFFu);
        for (uint32_t j = threadIdx.x; j < kCombBm; j += kCombThreads) L.bm[j] = 0ull;
        for (uint32_t j = threadIdx.x; j < kCombSlots; j += kCombThreads) {
            L.tab[j * 6] = 0ull;
#pragma unroll
            for (uint32_t w = 0; w < 4u; ++w) L.bytes[j * 4 + w] = 0ull;
#pragma unroll
            for (uint32_t w = 0; w < kCombF; ++w)
                L.f[j * kCombF + w] = (w == kCfFirst || w == kCfEnd || (w >= kCfChar && w < kCfChar + 4)) ? ~0u : 0u;
        }
        __syncthreads();
        K1CPH(1);
        // reduce per key (a key the table cannot take stays a plain entry), kCombU records per
        // thread at a time with their loads in flight together.  (Measured and not kept: four
        // records per thread, C4 Zipf(1.1) K1c 328 -> 415 us; a thread's consecutive records of
        // one key summed in registers before the LDS atomics, 328 -> 342 us.)
        for (uint32_t k0 = 0; k0 < cnt; k0 += kCombU * kCombThreads) {
            uint32_t wv[kCombU];
            uint4 rv[kCombU][4];
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u) {
                const uint32_t k = k0 + u * kCombThreads + threadIdx.x;
                wv[u] = k < cnt ? E[s0 + k] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u)
                if (k0 + u * kCombThreads + threadIdx.x < cnt) raw_entry(P, wv[u], rv[u]);
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u) {
                const uint32_t k = k0 + u * kCombThreads + threadIdx.x, w = wv[u];
                if (k >= cnt) continue;
                uint4 e[4];
                entry_of(P.ent != nullptr, rv[u], w, e);
                // the record's original word for the history (record order key | code: with update
                // entries rebuilt from the entry -- its pkt_index and character), read back by this
                // thread in the pack pass; its place in the chunk marked in the order bitmap
                const uint32_t eo = P.ent ? e[3].y | hist_code((e[3].z >> 16) & 1u, e[3].z & 0xFFu) << kEntCodeShift : w;
                P.e_orig[s0 + k] = eo;
                {
                    const uint32_t rc = (eo & kEntRecMask) - chunk * kFlowChunk;  // (< kFlowChunk, distinct)
                    if (rc < kFlowChunk) atomicOr(&L.bm[rc >> 6], 1ull << (rc & 63u));
                }
                const uint32_t key[10] = {e[0].x, e[0].y, e[0].z, e[0].w, e[1].x, e[1].y, e[1].z, e[1].w, e[2].x,
                                          e[2].y & 0xFFFFu};
                uint32_t j = lds_lookup<6, kCombSlots>(L.tab, key, e[3].w);
                const bool no_slot = j == ~0u && lds_upsert<6, kCombSlots>(L.tab, key, e[3].w, j) < 0;
                if (k < kCombJc) L.jc[k] = (no_slot || j >= 255u) ? 0xFFu : (uint8_t)j;
                if (no_slot) continue;
                const uint32_t orig = (e[2].y >> 16) & 1u, rec = e[3].y;
                uint32_t* f = L.f + j * kCombF;
                atomicAdd(&L.bytes[j * 4 + (orig ? 0u : 1u)], (unsigned long long)e[2].z);
                atomicAdd(&L.bytes[j * 4 + (orig ? 2u : 3u)], (unsigned long long)e[2].w);
                atomicAdd(f + kCfPk, orig ? 1u : 0x10000u);
                atomicAdd(f + kCfRecs, 1u);
                f[kCfHash] = e[3].w;  // every lane of the key stores the same word
                f[kCfMeta] = (e[3].z >> 20) & 0x1Fu;  // session flags + dst_service: a function of the key and the configuration
                atomicMin(f + kCfFirst, rec);
                const uint32_t psh = (e[3].z & 0x10000u) && ((e[3].z >> 8) & kTcpPsh) && (e[2].y & 0xFFu) == 6u ? 1u : 0u;
                atomicMax(f + kCfLast, rec << 1 | psh);  // (rec < 2^27) the last record and its PSH bit
                if (e[3].z & 0x10000u) {
                    atomicAdd(f + kCfHcnt, 1u | psh << 16);  // history count | PSH count << 16 (< kFlowChunk each)
                    const uint32_t b = hist_bit(e[3].z & 0xFFu);
                    if (b < 16u) atomicOr(f + kCfMask, 1u << b);
                    if (b < 4u) atomicMin(f + kCfChar + b, rec);
                    if ((e[3].z >> 8) & kTcpFinRst) atomicMin(f + kCfEnd, rec << 5 | b);  // (rec < 2^27)
                }
            }
        }
        __syncthreads();
        K1CPH(2);
        // number the keys met more than once; one global atomic per group for their ids
        constexpr uint32_t kPer = kCombSlots / kCombThreads;
        uint32_t nc = 0u;
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) nc += L.f[(threadIdx.x * kPer + u) * kCombF + kCfRecs] >= 2u;
        uint32_t n_comb;
        uint32_t rank = block_excl_scan(nc, L.wsum, n_comb);
        if (n_comb == 0u) continue;  // uniform across the block; the table is re-initialised above
        if (threadIdx.x == 0) {
            uint32_t nx = L.pool_next, en = L.pool_end;
            if (en - nx < n_comb) {
                const uint32_t g = max(n_comb, pool);
                nx = atomicAdd(P.ctl + 1, g);
                en = nx + g;
            }
            L.base = nx;
            L.pool_next = nx + n_comb;
            L.pool_end = en;
        }
        __syncthreads();
        K1CPH(3);
        const uint32_t id0 = L.base;
        if (id0 + n_comb > P.comb_cap) continue;  // no room for its combined entries: the group stays plain
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
            uint32_t* f = L.f + (threadIdx.x * kPer + u) * kCombF;
            if (f[kCfRecs] >= 2u) f[kCfId] = rank++;
        }
        {   // the order bitmap's prefix popcounts (thread t: words kCombBmPer t ..)
            const uint32_t w0 = kCombBmPer * threadIdx.x;
            uint32_t c[kCombBmPer], sum = 0u;
#pragma unroll
            for (uint32_t u = 0; u < kCombBmPer; ++u) {
                c[u] = w0 + u < kCombBm ? (uint32_t)__popcll(L.bm[w0 + u]) : 0u;
                sum += c[u];
            }
            uint32_t tot;
            uint32_t ex = block_excl_scan(sum, L.wsum, tot);
#pragma unroll
            for (uint32_t u = 0; u < kCombBmPer; ++u) {
                if (w0 + u < kCombBm) L.bmp[w0 + u] = (uint16_t)ex;
                ex += c[u];
            }
        }
        __syncthreads();
        K1CPH(4);
        // pack the remaining plain entries (record indices) to the front, tile by tile of kCombU
        // records per thread (a tile is loaded before any of its stores, and stores land below the
        // next tile); every record's original word and new position (combined id or moved entry)
        // go to e_sort at its rank
        uint32_t cursor = 0u;
        for (uint32_t t = 0; t < cnt; t += kCombU * kCombThreads) {
            uint32_t rec[kCombU], eo[kCombU], v[kCombU], nk = 0u;
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u) {
                const uint32_t k = t + u * kCombThreads + threadIdx.x;
                rec[u] = k < cnt ? E[s0 + k] : 0u;
                eo[u] = k < cnt ? P.e_orig[s0 + k] : 0u;  // (this thread's own store of the reduce pass)
            }
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u) {
                const uint32_t k = t + u * kCombThreads + threadIdx.x;
                v[u] = ~0u;  // ~0: kept (its new position follows the scan)
                if (k >= cnt) continue;
                uint32_t j = k < kCombJc ? L.jc[k] : 0xFFu;
                if (j == 0xFFu) {  // past the cache, no slot, or slot 255: find the key again
                    uint4 e[4];
                    rec_entry(P, rec[u], e);
                    const uint32_t key[10] = {e[0].x, e[0].y, e[0].z, e[0].w, e[1].x, e[1].y, e[1].z, e[1].w, e[2].x,
                                              e[2].y & 0xFFFFu};
                    j = lds_find<6, kCombSlots>(L.tab, key, e[3].w);
                }
                if (j != ~0u && L.f[j * kCombF + kCfRecs] >= 2u) v[u] = kRecFlowCombined | (id0 + L.f[j * kCombF + kCfId]);
                else ++nk;
            }
            uint32_t kept;
            uint32_t pos = cursor + block_excl_scan(nk, L.wsum, kept);
#pragma unroll
            for (uint32_t u = 0; u < kCombU; ++u) {
                const uint32_t k = t + u * kCombThreads + threadIdx.x;
                if (k >= cnt) continue;
                if (v[u] == ~0u) {
                    v[u] = (uint32_t)(s0 + pos);  // the entry moved
                    E[s0 + pos] = rec[u];
                    ++pos;
                }
                const uint32_t rc = min((eo[u] & kEntRecMask) - chunk * kFlowChunk, kFlowChunk - 1u);
                const uint32_t rank = L.bmp[rc >> 6] + (uint32_t)__popcll(L.bm[rc >> 6] & ((1ull << (rc & 63u)) - 1ull));
                P.e_sort[s0 + min(rank, cnt - 1u)] = make_uint2(eo[u], v[u]);
            }
            cursor += kept;
        }
        K1CPH(5);
        // the combined entries (two units each in P.comb) and their index words behind the kept ones
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
            const uint32_t j = threadIdx.x * kPer + u;
            const uint32_t* f = L.f + j * kCombF;
            if (f[kCfRecs] < 2u) continue;
            const uint32_t id = id0 + f[kCfId];
            const unsigned long long* tw = L.tab + j * 6;
            const unsigned long long* by = L.bytes + j * 4;
            uint4* o = CE + (size_t)id * 8u;
            o[0] = make_uint4((uint32_t)tw[1], (uint32_t)(tw[1] >> 32), (uint32_t)tw[2], (uint32_t)(tw[2] >> 32));
            o[1] = make_uint4((uint32_t)tw[3], (uint32_t)(tw[3] >> 32), (uint32_t)tw[4], (uint32_t)(tw[4] >> 32));
            o[2] = make_uint4((uint32_t)tw[5], (uint32_t)(tw[5] >> 32) | kEntCombined, f[kCfFirst], f[kCfLast] >> 1);
            o[3] = make_uint4(id, f[kCfEnd] == ~0u ? ~0u : f[kCfEnd] >> 5, (f[kCfHcnt] & 0xFFFFu) | (f[kCfMask] << 16), f[kCfHash]);
            o[4] = make_uint4((uint32_t)by[0], (uint32_t)(by[0] >> 32), (uint32_t)by[1], (uint32_t)(by[1] >> 32));
            o[5] = make_uint4((uint32_t)by[2], (uint32_t)(by[2] >> 32), (uint32_t)by[3], (uint32_t)(by[3] >> 32));
            o[6] = make_uint4(f[kCfPk], kEntTail, f[kCfChar], f[kCfChar + 1]);
            o[7] = make_uint4(f[kCfChar + 2], f[kCfChar + 3], f[kCfRecs],
                              f[kCfMeta] | (f[kCfEnd] & 31u) << 8 | (f[kCfLast] & 1u) << 15 | (f[kCfHcnt] >> 16) << 16);
            E[s0 + cursor + f[kCfId]] = kIdxCombined | id;
        }
        if (threadIdx.x == 0) {  // bit 15: a combined group (the history reads e_sort, and
                                 // the group's original row from rows_h)
            *rowp = (row & 0x7FFFu) | 0x8000u | ((cursor + n_comb) << 16);
            P.rows_h[(size_t)chunk * P.parts + part] = row;
        }
        __syncthreads();  // the table is re-initialised for the next group
        K1CPH(6);
    }
#undef K1CPH
    FLOWTR(if (threadIdx.x == 0 && blockIdx.x < 1024u) {
        unsigned long long* t = g_k1c_trace + kK1cTrWords * blockIdx.x;
        t[0] = tr_t0;
        t[1] = flow_now();
        t[2] = tr_groups;
        t[3] = tr_recs;
        for (uint32_t k = 0; k < 7u; ++k) t[4 + k] = tr_ph[k];
        t[11] = 0ull;
    });
}

__global__ __launch_bounds__(kFlowK2Threads, 2 * kFlowK2Threads / 256) void k_flow_apply(const FlowParams P) {
    extern __shared__ uint4 slice4[];  // kFlowSlots 96-B slot heads, then kFlowSlots 40-B scratch
    __shared__ uint32_t sp[kK2Cpt * kFlowK2Threads];
    __shared__ uint32_t ss[kK2Cpt * kFlowK2Threads];
    __shared__ uint32_t wsum[kFlowK2Threads / 64];
    __shared__ unsigned long long sh[kFlowK2Threads / 64];
    __shared__ uint32_t s_hbase;
    unsigned long long* slice = reinterpret_cast<unsigned long long*>(slice4);
    uint32_t* scr = reinterpret_cast<uint32_t*>(slice + (size_t)kFlowSlots * kSlotWords);
    uint32_t* tags = scr + (size_t)kFlowSlots * kScrU32;  // FB_K2_TAGS: the slots' probe tags
    // the leading workgroups take the partitions with the most entries (K1t's list), the rest the
    // other partitions in order; the grid has kK2Lead workgroups more than partitions with P.order
    // (a later workgroup's check of its partition waits below, behind its first loads)
    uint32_t part = blockIdx.x, led = 0u;
    if (P.order) {
        if (blockIdx.x < kK2Lead) {
            if (blockIdx.x >= min(P.order[P.parts + kK2Lead], kK2Lead)) return;  // (uniform)
            part = P.order[P.parts + blockIdx.x];
        } else {
            part = blockIdx.x - kK2Lead;
            led = P.order[part];
        }
    }
    const uint32_t n = batch_records(P);
    const uint32_t chunks = (n + kFlowChunk - 1u) / kFlowChunk;
    const uint32_t* col = P.cols + (size_t)part * P.chunk_stride;
#ifdef FB_FLOW_TRACE
    const unsigned long long tr_t0 = flow_now();
    unsigned long long tr_t1 = 0ull;
    __shared__ uint32_t tr_hmax;
    if (threadIdx.x == 0) tr_hmax = 0u;
#endif

    // the first round's group rows (kept for it) and the rows past it: the partition's total
    uint32_t v0[kK2Cpt], mine = 0u;
#pragma unroll
    for (uint32_t c = 0; c < kK2Cpt; ++c) {
        const uint32_t b = threadIdx.x * kK2Cpt + c;
        v0[c] = b < chunks ? col[b] : 0u;
        mine += v0[c] >> 16;
    }
    for (uint32_t b = kK2Cpt * kFlowK2Threads + threadIdx.x; b < chunks; b += kFlowK2Threads) mine += col[b] >> 16;
    constexpr uint32_t kHead16 = kSlotWords * 8u / 16u;  // 6 uint4 per slot head
    FlowSlot* T = P.table + (size_t)part * kFlowSlots;
    const uint4* g = reinterpret_cast<const uint4*>(T);
    // the slice heads into LDS and slot tid's ordered fields (for finish_slot) into registers
    static_assert(kFlowSlots == kFlowK2Threads, "one slot per thread in the fold");
    uint4 ord0, ord1;
    uint32_t tag0 = 0u;  // slot tid's tag, low word
    auto load_slice = [&]() {
        ord0 = g[(size_t)threadIdx.x * 8u + 6u];
        ord1 = g[(size_t)threadIdx.x * 8u + 7u];
        if (FB_K2_TAGS) tag0 = reinterpret_cast<const uint32_t*>(g + (size_t)threadIdx.x * 8u)[0];
        for (uint32_t j = threadIdx.x; j < kFlowSlots * kHead16; j += kFlowK2Threads) {
            const uint32_t sl = j / kHead16, w = j - sl * kHead16;
            slice4[j] = g[(size_t)sl * (sizeof(FlowSlot) / 16u) + w];
        }
    };
    // a batch with >= 32 record slots per partition touches nearly every partition: the slice
    // load is issued with the group rows, before the partition's total is known (one round trip
    // less per workgroup); sparser batches load it only for a partition with entries
#ifndef FB_K2_PREFETCH
#define FB_K2_PREFETCH 1
#endif
    const bool dense = FB_K2_PREFETCH && n >= 32u * P.parts;
    // (uniform) a leading workgroup's partition: leave before its 64-KB slice is loaded a second
    // time (the order word was issued before the group rows, so this waits for it alone)
    if (led >> 31) return;
    if (dense) load_slice();
    const unsigned long long total = block_sum(mine, sh);
    unsigned long long n_new = 0ull, n_upd = 0ull;
    uint32_t hbase_out = 0u, hc = 0u;
    if (total != 0ull) {
        if (!dense) load_slice();
        for (uint32_t j = threadIdx.x; j < kFlowSlots * kScrU32; j += kFlowK2Threads) {
            const uint32_t w = j % kScrU32;
            scr[j] = (w == kScLast || w == kScLast + 1u || w == kScMask || w == kScCount) ? 0u : ~0u;
        }
        if (FB_K2_TAGS) tags[threadIdx.x] = tag0;
        if (threadIdx.x == 0) s_hbase = atomicAdd(P.ctl + 2, (uint32_t)total);  // the history words' range
        __syncthreads();
        const uint32_t hbase = s_hbase;
        hbase_out = hbase;
        uint32_t rbase = 0u;  // entries of the earlier rounds
        const uint32_t* E = P.entries;
        const uint4* CE = reinterpret_cast<const uint4*>(P.comb);
        for (uint32_t g0 = 0; g0 < chunks; g0 += kK2Cpt * kFlowK2Threads) {
            // kK2Cpt consecutive chunks per thread: one round for batches up to kK2Cpt x 512 chunks
            uint32_t v[kK2Cpt], mine = 0u;
#pragma unroll
            for (uint32_t c = 0; c < kK2Cpt; ++c) {
                const uint32_t b = g0 + threadIdx.x * kK2Cpt + c;
                v[c] = g0 == 0u ? v0[c] : (b < chunks ? col[b] : 0u);
                mine += v[c] >> 16;
            }
            uint32_t tot;
            uint32_t pre = block_excl_scan(mine, wsum, tot);
#pragma unroll
            for (uint32_t c = 0; c < kK2Cpt; ++c) {
                const uint32_t j = threadIdx.x * kK2Cpt + c;
                sp[j] = pre;
                ss[j] = (g0 + j) * kFlowChunk + (v[c] & 0x7FFFu);  // (bit 15: combined group)
                pre += v[c] >> 16;
            }
            __syncthreads();
            // Entries of this round, software-pipelined per thread (entries e, e+S, e+2S, ... of
            // thread e: consecutive lanes read consecutive index words): the index word of entry
            // e+2S and the record (or combined entry) of e+S are in flight while entry e is applied
            // (each entry otherwise waits two dependent memory round trips: its index, then its
            // record).  Contiguous per-thread runs with a forward walk instead of the per-entry
            // binary search measured slower (C4 K2 672 -> 808 us).
            constexpr uint32_t S = kFlowK2Threads;
            auto locate = [&](uint32_t e) {  // entry position of round entry e: largest j with sp[j] <= e
                uint32_t lo = 0u, hi = kK2Cpt * kFlowK2Threads - 1u;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1u) >> 1;
                    if (sp[mid] <= e) lo = mid; else hi = mid - 1u;
                }
                return ss[lo] + (e - sp[lo]);
            };
            auto gather = [&](uint32_t v, uint4 (&r)[4]) {  // raw words only; decoded when applied
                if (v & kIdxCombined) {  // a k_flow_combine entry: head unit (the tail is read when applied)
                    const uint4* c = CE + (size_t)(v & ~kIdxCombined) * 8u;
                    r[0] = c[0];
                    r[1] = c[1];
                    r[2] = c[2];
                    r[3] = c[3];
                } else {  // a record slot of the batch: its update entry or its record
                    raw_entry(P, v, r);
                }
            };
            uint32_t e = threadIdx.x, ix0 = 0u, v0 = 0u, ix1 = 0u, v1 = 0u;
            uint4 r0[4], r1[4];
            if (e < tot) {
                ix0 = locate(e);
                v0 = E[ix0];
            }
            if (e + S < tot) {
                ix1 = locate(e + S);
                v1 = E[ix1];
            }
            if (e < tot) gather(v0, r0);
            for (; e < tot; e += S) {
                uint32_t ix2 = 0u, v2 = 0u;
                if (e + 2u * S < tot) {
                    ix2 = locate(e + 2u * S);
                    v2 = E[ix2];
                }
                if (e + S < tot) gather(v1, r1);
                if (v0 & kIdxCombined) {
                    const uint4* t = CE + (size_t)(v0 & ~kIdxCombined) * 8u + 4u;
                    const uint4 t3 = t[3];
                    const int r = apply_combined(slice, tags, scr, P, r0[0], r0[1], r0[2], r0[3], t[0], t[1], t[2], t3,
                                                 part * kFlowSlots, P.agg_slot, P.error);
                    if (r >= 0) {
                        n_new += r == 1;
                        n_upd += t3.z - (r == 1 ? 1u : 0u);
                    }
                } else {
                    // the entry as a plain FlowEntry (layout: fb_internal.h; entry_of above)
                    uint4 fe[4];
                    entry_of(P.ent != nullptr, r0, v0, fe);
                    uint32_t sl = ~0u;
                    const int r = apply_entry(slice, tags, scr, fe[0], fe[1], fe[2], fe[3], sl, P.error);
                    n_new += r == 1;
                    n_upd += r == 0;
                    // the history word (layout: fb_internal.h), in this partition's entry order
                    // (with update entries the code comes from the entry and rec is its pkt_index)
                    P.hword[hbase + rbase + e] =
                        r < 0 ? 0u
                              : P.ent ? hist_word(sl, hist_code((fe[3].z >> 16) & 1u, fe[3].z & 0xFFu), fe[3].y)
                                      : hist_word(sl, v0);
                    if (P.tkv) {  // timed contexts: the capture-time pass's sort input at the record slot
                        // (an update entry's record slot: its segment's 64 slots + its rank, unit 0 word 7):
                        // table slot << 32 | pkt_index << 1 | PSH (TCP with flags)
                        const uint32_t rs = P.ent ? ((v0 & kEntUnitMask) / kUpdUnitsPerSeg) * 64u + (r0[1].w >> 26)
                                                  : (v0 & kEntRecMask);
                        const uint32_t hi = fe[3].z;  // hist_char | tcp_flags << 8 | has_flags << 16
                        const bool psh = ((hi >> 16) & 1u) && (fe[2].y & 0xFFu) == 6u && ((hi >> 8) & kTcpPsh);
                        P.tkv[rs] = (unsigned long long)(r < 0 ? ~0u : part * kFlowSlots + sl) << 32 |
                                    (fe[3].x << 1 | (psh ? 1u : 0u));
                    }
                }
#pragma unroll
                for (uint32_t w = 0; w < 4u; ++w) r0[w] = r1[w];
                ix0 = ix1;
                v0 = v1;
                ix1 = ix2;
                v1 = v2;
            }
            rbase += tot;
            __syncthreads();
        }
        hc = scr[(size_t)threadIdx.x * kScrU32 + kScCount];  // (before the fold reuses the word)
        FLOWTR(tr_t1 = flow_now(); atomicMax(&tr_hmax, hc));
        finish_slot(scr + (size_t)threadIdx.x * kScrU32, P.batch, ord0, ord1,
                    P.char_call ? P.char_call + (size_t)part * kFlowSlots + threadIdx.x : nullptr);
        __syncthreads();  // every slot's new ordered fields are in its scratch
        // only the slots this batch touched (inserted or updated) changed; each is written back as
        // one whole 128-B line (head from the slice, ordered fields from the scratch): eight
        // consecutive lanes per slot, so a wavefront stores eight full lines
        uint4* gw = reinterpret_cast<uint4*>(T);
        constexpr uint32_t kSlot16 = sizeof(FlowSlot) / 16u;  // 8
        for (uint32_t j = threadIdx.x; j < kFlowSlots * kSlot16; j += kFlowK2Threads) {
            const uint32_t sl = j / kSlot16, w = j - sl * kSlot16;
            const uint32_t* q = scr + (size_t)sl * kScrU32;
            if (q[kScFirst + 1u] != ~0u)  // the first key's rec word: touched
                gw[j] = w < kHead16 ? slice4[(size_t)sl * kHead16 + w]
                                    : reinterpret_cast<const uint4*>(q + kScOrd)[w - kHead16];
        }
    }
    n_new = block_sum(n_new, sh);
    n_upd = block_sum(n_upd, sh);
    // occupied slots after the update (the host grows the table from these, k_flow_finish)
    unsigned long long occ = total != 0ull ? (FB_K2_TAGS ? tags[threadIdx.x] >= 2u : slice[(size_t)threadIdx.x * kSlotWords] >= 2ull)
                                           : g[(size_t)threadIdx.x * 8u].x >= 2u;
    occ = block_sum(occ, sh);
    // history characters per slot this update (the history's output offsets), and their total
    P.hcount[(size_t)part * kFlowSlots + threadIdx.x] = hc;
    const unsigned long long hcs = block_sum((unsigned long long)hc, sh);
    FLOWTR(if (threadIdx.x == 0 && part < kFlowTrParts) {
        unsigned long long* t = g_k2_trace + 4u * part;
        t[0] = tr_t0;
        t[1] = tr_t1;
        t[2] = flow_now();
        t[3] = total | (unsigned long long)tr_hmax << 32;
    });
    if (threadIdx.x == 0) {
        P.partials[4 * part] = n_new;
        P.partials[4 * part + 1] = n_upd;
        P.partials[4 * part + 2] = occ;
        P.partials[4 * part + 3] = hcs | (unsigned long long)hbase_out << 32;
    }
}

__global__ __launch_bounds__(1024) void k_flow_finish(fb_batch_stats* S, const unsigned long long* part,
                                                      uint32_t nblk, const uint32_t* err, FlowMailbox* mbox,
                                                      unsigned long long seq) {
    __shared__ unsigned long long sh[16];
    unsigned long long a = 0ull, b = 0ull, o = 0ull, m = 0ull;
    for (uint32_t i = threadIdx.x; i < nblk; i += blockDim.x) {
        a += part[4 * i];
        b += part[4 * i + 1];
        o += part[4 * i + 2];
        m = max(m, part[4 * i + 2]);
    }
    a = block_sum(a, sh);
    b = block_sum(b, sh);
    o = block_sum(o, sh);
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, k, 64));
    if ((threadIdx.x & 63u) == 0u) sh[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < blockDim.x / 64u; ++w) m = max(m, sh[w]);
        S->new_sessions += a;
        S->updated_sessions += b;
        S->error |= *err;
        if (mbox) {  // host-mapped: the occupancy first, the sequence number last (system-scope stores)
            __hip_atomic_store(&mbox->flows, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mbox->max_part, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mbox->new_flows, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mbox->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Growth by 2^k: old partition p (one workgroup, one slot per thread) splits into new partitions
// p * 2^k .. p * 2^k + 2^k - 1 (the next k top bits of the key's hash); each key is re-inserted from
// its unchanged home slot (low bits of the hash) by linear probing, the claim made on an LDS array
// per new partition.
__global__ __launch_bounds__(kFlowSlots) void k_flow_grow(const FlowSlot* old, uint32_t new_shift, uint32_t k,
                                                          FlowSlot* nw, uint32_t* remap, const uint4* old_cc,
                                                          uint4* new_cc) {
    extern __shared__ uint32_t claim_w[];  // [2^k][kFlowSlots]
    const uint32_t p = blockIdx.x, i = threadIdx.x;
    for (uint32_t j = i; j < (kFlowSlots << k); j += kFlowSlots) claim_w[j] = 0u;
    __syncthreads();
    const FlowSlot& o = old[(size_t)p * kFlowSlots + i];
    uint32_t dst = ~0u;
    if (o.tag >= 2ull) {
        uint32_t key[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) key[k] = o.key[k];
        const unsigned long long h = flow_hash_words(key);
        const uint32_t b = new_shift >= 64u ? 0u : (uint32_t)(h >> new_shift) & ((1u << k) - 1u);
        uint32_t* claim = claim_w + b * kFlowSlots;
        uint32_t j = (uint32_t)h & (kFlowSlots - 1u);
        while (atomicCAS(&claim[j], 0u, 1u) != 0u) j = (j + 1u) & (kFlowSlots - 1u);  // a partition holds <= 512 keys
        dst = ((p << k) + b) * kFlowSlots + j;
        const uint4* src = reinterpret_cast<const uint4*>(&o);
        uint4* d = reinterpret_cast<uint4*>(nw + dst);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = src[k];
        if (old_cc) new_cc[dst] = old_cc[(size_t)p * kFlowSlots + i];
    }
    remap[(size_t)p * kFlowSlots + i] = dst;
}

// is_local_session! (src/sessions.rs:660-666) of a slot's key under the current configuration.
__device__ __forceinline__ bool slot_local(const DevConfig* cfg, const FlowSlot& t) {
    const uint32_t fam = (t.key[9] >> 8) & 0xFFu;
    if (fam == 2u) return lan_v4(t.key[0]) && lan_v4(t.key[4]);
    const uint32_t s[4] = {t.key[0], t.key[1], t.key[2], t.key[3]}, d[4] = {t.key[4], t.key[5], t.key[6], t.key[7]};
    return lan_v6(cfg, cfg, s) && lan_v6(cfg, cfg, d);
}

__global__ __launch_bounds__(256) void k_flow_export(const FlowSlot* T, unsigned long long cap,
                                                     fb_flow_rec* out, unsigned long long out_cap,
                                                     unsigned long long* d_n, uint32_t filter, const DevConfig* cfg,
                                                     const FlowTime* plane) {
    __shared__ unsigned long long sh[4];
    __shared__ unsigned long long s_base;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < cap; base += stride) {
        const unsigned long long i = base + threadIdx.x;
        bool occ = i < cap && T[i].tag >= 2ull;
        // get_sessions' read-time filter (src/capture.rs:1603-1608): is_lan_ip evaluated now
        if (occ && filter != FB_FILTER_ALL) occ = slot_local(cfg, T[i]) == (filter == FB_FILTER_LOCAL_ONLY);
        const unsigned long long m = __ballot(occ);
        const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
        if (lane == 0u) sh[wave] = __popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long tot = sh[0] + sh[1] + sh[2] + sh[3];
            s_base = tot ? atomicAdd(d_n, tot) : 0ull;
        }
        __syncthreads();
        unsigned long long pos = s_base + __popcll(m & ((1ull << lane) - 1ull));
        for (uint32_t w = 0; w < wave; ++w) pos += sh[w];
        if (occ && pos < out_cap) {
            fb_flow_rec r = flow_rec_of(T[i], (uint32_t)i);
            if (plane) {  // a timed context: the segment state with the 5-s timeout (fb_time.hip)
                r.segment_count = plane[i].segment_count;
                r.in_segment = plane[i].in_segment;
            }
            out[pos] = r;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_flow_count(const FlowSlot* T, unsigned long long cap,
                                                    unsigned long long* d_n) {
    __shared__ unsigned long long sh[4];
    unsigned long long c = 0ull;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride)
        c += T[i].tag >= 2ull;
    c = block_sum(c, sh);
    if (threadIdx.x == 0 && c) atomicAdd(d_n, c);
}

hipError_t launch_flow_combine(const FlowParams& p, hipStream_t s) {
    if (!p.hot) return hipSuccess;
    hipLaunchKernelGGL(k_flow_combine, dim3(kCombGrid), dim3(kCombThreads), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_flow_bucket(const FlowParams& p, uint32_t chunks, hipStream_t s, bool combine) {
    if (chunks == 0u) chunks = 1u;
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)k_flow_bucket, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)std::max(k1_lds_bytes(kFlowMaxParts), k1_lds_bytes(kFlowPackedParts)));
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(k_flow_bucket, dim3(chunks), dim3(kFlowK1Threads), k1_lds_bytes(p.parts), s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return combine ? launch_flow_combine(p, s) : e;
}
hipError_t launch_flow_transpose(const FlowParams& p, uint32_t chunks, hipStream_t s) {
    if (chunks == 0u) chunks = 1u;
    hipLaunchKernelGGL(k_flow_transpose, dim3((p.parts + 63u) / 64u, (chunks + 63u) / 64u), dim3(256), 0, s, p,
                       chunks);
    return hipGetLastError();
}
hipError_t launch_flow_apply(const FlowParams& p, uint32_t chunks, hipStream_t s, bool transpose) {
    if (transpose) {
        const hipError_t e = launch_flow_transpose(p, chunks, s);
        if (e != hipSuccess) return e;
    }
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k_flow_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kK2Lds);
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(k_flow_apply, dim3(p.parts + (p.order ? kK2Lead : 0u)), dim3(kFlowK2Threads), kK2Lds, s, p);
    return hipGetLastError();
}
hipError_t launch_flow_finish(fb_batch_stats* stats, const unsigned long long* partials, uint32_t nblk,
                              uint32_t* error, FlowMailbox* mbox, unsigned long long seq, hipStream_t s) {
    hipLaunchKernelGGL(k_flow_finish, dim3(1), dim3(1024), 0, s, stats, partials, nblk, error, mbox, seq);
    return hipGetLastError();
}
hipError_t launch_flow_grow(const FlowSlot* old, uint32_t old_parts, uint32_t k, uint32_t new_shift, FlowSlot* nw,
                            uint32_t* remap, const uint4* old_cc, uint4* new_cc, hipStream_t s) {
    if (k < 1u || k > 5u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_flow_grow, dim3(old_parts), dim3(kFlowSlots), (kFlowSlots << k) * 4u, s, old, new_shift, k, nw,
                       remap, old_cc, new_cc);
    return hipGetLastError();
}
hipError_t launch_flow_export(const FlowSlot* table, unsigned long long cap, fb_flow_rec* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s, uint32_t filter,
                              const DevConfig* cfg, const FlowTime* plane) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > 1024ull) g = 1024ull;
    if (g == 0ull) g = 1ull;
    if (!cfg) filter = FB_FILTER_ALL;
    hipLaunchKernelGGL(k_flow_export, dim3((uint32_t)g), dim3(256), 0, s, table, cap, out, out_cap, d_n, filter, cfg,
                       plane);
    return hipGetLastError();
}
hipError_t launch_flow_count(const FlowSlot* table, unsigned long long cap, unsigned long long* d_n,
                             hipStream_t s) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > 1024ull) g = 1024ull;
    if (g == 0ull) g = 1ull;
    hipLaunchKernelGGL(k_flow_count, dim3((uint32_t)g), dim3(256), 0, s, table, cap, d_n);
    return hipGetLastError();
}

}  // namespace fbk

#ifdef FB_FLOW_TRACE
// diagnostic builds only: the last K2 launch's per-partition trace (4 x 8192 words), then the last
// K1c launch's per-workgroup trace (12 x 1024 words), after a device sync
extern "C" __attribute__((visibility("default"))) int fb_flow_trace_last(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fbk::g_k2_trace), sizeof(fbk::g_k2_trace)) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out + 4u * fbk::kFlowTrParts, HIP_SYMBOL(fbk::g_k1c_trace),
                               sizeof(fbk::g_k1c_trace)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" uint64_t fb_flow_hash(const fb_session_key* key) {
    uint32_t w[10];
    __builtin_memcpy(w, key, 40);
    w[9] &= 0xFFFFu;  // the key's padding is not part of the key
    return fbk::flow_hash_words(w);
}
