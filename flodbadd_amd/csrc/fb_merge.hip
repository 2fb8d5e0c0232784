// fb_merge.hip -- gfx950 kernels of the multi-GPU session-table merge (BASELINE configs[4]).
//
// The reference keeps ONE session map that every capture task updates (src/capture.rs:946-1016,
// src/packets.rs:329-535).  Here W ranks each build a table from a contiguous packet-index shard
// (flodbadd_amd/distributed.py moves the records between ranks with RCCL); these kernels are the
// two local steps around that exchange:
//   export  every flow of a rank's table as an fb_flow_mrec, grouped by owner rank (flow_owner of
//           its hash), slot order inside a group, positions made global (+ the shard's first packet
//           index), rec.slot = the rank, and the update call of the flow's first S / s / H / h;
//   merge   the records one owner received (each rank's group, rank order) -> one record per key:
//           integer counter sums (segment_count too), MIN first_seen, MAX last_seen, hist_len SUM,
//           hist_mask OR, in_segment of the record holding the latest packet and the session flags
//           of the one holding the earliest (the flow's insert: src/packets.rs:429-466), and
//           the ordered state at the GLOBAL first FIN/RST (src/packets.rs:187-198, 422-426,
//           539-559): end_seen = the smallest end over the ranks; end_mask = the ending rank's own
//           end_mask (the characters its history held at that packet) OR, for every other rank, the
//           S s H h whose first occurrence precedes the end packet in global order -- an earlier
//           update call, or the same call on a lower rank (global batch k = the ranks' k-th shards
//           in rank order); F f R r come only from FIN/RST packets, and the first of those IS the
//           end packet.  conn_state = determine_conn_state over that set.
// Every reduction is a sum / min / max / or, so the result does not depend on the order in which
// the atomics land; each key's record is placed at the position of its first input record (a
// prefix sum over "first record of its key" flags), so the output order is deterministic too.
#include <algorithm>

#include "fb_internal.h"

namespace fbk {

// ---------------------------------------------------------------------------------------------
// Export.  One wavefront per chunk of kMxChunk slots: pass 1 counts each owner's flows per chunk,
// a single-workgroup scan turns the counts into owner-major offsets, pass 2 writes each chunk's
// flows owner by owner in slot order (one ballot per owner and 64-slot step).
constexpr uint32_t kMxChunk = 4096;
constexpr uint32_t kMxMaxWorld = 64;

__device__ __forceinline__ bool slot_occupied(const FlowSlot* T, unsigned long long i, unsigned long long cap) {
    return i < cap && T[i].tag >= 2ull;
}
__device__ __forceinline__ uint32_t slot_owner(const FlowSlot& t, uint32_t world) {
    uint32_t key[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) key[k] = t.key[k];
    key[9] &= 0xFFFFu;
    return flow_owner(flow_hash_words(key), world);
}

__global__ __launch_bounds__(64) void k_mx_count(const FlowSlot* T, unsigned long long cap, uint32_t world,
                                                 uint32_t* cnt /* [chunks][world] */) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long c0 = (unsigned long long)blockIdx.x * kMxChunk;
    uint32_t mine = 0u;  // lane o: owner o's flows in this chunk
    for (uint32_t j = 0; j < kMxChunk; j += 64u) {
        const unsigned long long i = c0 + j + lane;
        const bool occ = slot_occupied(T, i, cap);
        const uint32_t o = occ ? slot_owner(T[i], world) : ~0u;
        for (uint32_t w = 0; w < world; ++w) {
            const uint32_t k = (uint32_t)__popcll(__ballot(o == w));
            if (lane == w) mine += k;
        }
    }
    if (lane < world) cnt[(size_t)blockIdx.x * world + lane] = mine;
}

// Exclusive scan of one u32 per thread over a workgroup (blockDim a multiple of 64, <= 1024).
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* ws, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63u) ws[wave] = x;
    __syncthreads();
    uint32_t before = 0u, tot = 0u;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint32_t t = ws[w];
        before += w < wave ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

// cnt[chunk][owner] -> off[chunk][owner] = (flows of lower owners) + (the owner's flows in earlier
// chunks); d_counts[owner] = the owner's flows.  One 1024-thread workgroup, owner by owner, each
// thread scanning a contiguous run of chunks.
__global__ __launch_bounds__(1024) void k_mx_scan(uint32_t* cnt, uint32_t chunks, uint32_t world,
                                                  unsigned long long* d_counts) {
    __shared__ uint32_t ws[16];
    const uint32_t per = (chunks + 1023u) / 1024u, c0 = threadIdx.x * per, c1 = min(c0 + per, chunks);
    uint32_t base = 0u;
    for (uint32_t o = 0; o < world; ++o) {
        uint32_t s = 0u;
        for (uint32_t c = c0; c < c1; ++c) s += cnt[(size_t)c * world + o];
        uint32_t tot;
        uint32_t run = base + wg_excl_scan(s, ws, tot);
        for (uint32_t c = c0; c < c1; ++c) {
            const uint32_t v = cnt[(size_t)c * world + o];
            cnt[(size_t)c * world + o] = run;
            run += v;
        }
        if (threadIdx.x == 0) d_counts[o] = tot;
        base += tot;
    }
}

// A table position (update call << 32 | pkt_index) made global: with a call map, call k of this rank
// was its shard of global batch cmap[k] >> 32 starting at global packet cmap[k] & 0xFFFFFFFF; without
// one, call k is global batch k with the shard at shard_first in each.
__device__ __forceinline__ unsigned long long global_pos(unsigned long long p, unsigned long long shard_first,
                                                         const unsigned long long* cmap) {
    const unsigned long long lo = 0xFFFFFFFFull;
    const unsigned long long m = cmap ? cmap[p >> 32] : ((p & ~lo) | shard_first);
    return (m & ~lo) | ((m & lo) + (p & lo));
}

__global__ __launch_bounds__(64) void k_mx_write(const FlowSlot* T, const uint4* cc, unsigned long long cap,
                                                 uint32_t world, uint32_t rank, unsigned long long shard_first,
                                                 const unsigned long long* cmap, const uint32_t* off,
                                                 fb_flow_mrec* out, unsigned long long out_cap) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long c0 = (unsigned long long)blockIdx.x * kMxChunk;
    uint32_t next = lane < world ? off[(size_t)blockIdx.x * world + lane] : 0u;  // lane o: owner o's cursor
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t j = 0; j < kMxChunk; j += 64u) {
        const unsigned long long i = c0 + j + lane;
        const bool occ = slot_occupied(T, i, cap);
        const uint32_t o = occ ? slot_owner(T[i], world) : ~0u;
        uint32_t pos = 0u;
        for (uint32_t w = 0; w < world; ++w) {
            const unsigned long long m = __ballot(o == w);
            const uint32_t base = (uint32_t)__shfl((int)next, (int)w, 64);
            if (o == w) pos = base + (uint32_t)__popcll(m & lt);
            if (lane == w) next += (uint32_t)__popcll(m);
        }
        if (occ && pos < out_cap) {
            fb_flow_mrec r;
            r.rec = flow_rec_of(T[i], rank);
            // positions (call << 32 | pkt_index) -> (global batch << 32 | global packet index); end
            // None stays None; the calls of the first S s H h -> their global batches
            r.rec.first_seen = global_pos(r.rec.first_seen, shard_first, cmap);
            r.rec.last_seen = global_pos(r.rec.last_seen, shard_first, cmap);
            if (r.rec.end_seen != FB_SEEN_NONE) r.rec.end_seen = global_pos(r.rec.end_seen, shard_first, cmap);
            const uint4 c = cc ? cc[i] : make_uint4(FB_CALL_NONE, FB_CALL_NONE, FB_CALL_NONE, FB_CALL_NONE);
            const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int b = 0; b < 4; ++b)
                r.char_call[b] = (cw[b] == FB_CALL_NONE || !cmap) ? cw[b] : (uint32_t)(cmap[cw[b]] >> 32);
            out[pos] = r;
        }
    }
}

uint64_t merge_export_scratch_bytes(unsigned long long cap, uint32_t world) {
    const unsigned long long chunks = (cap + kMxChunk - 1) / kMxChunk;
    return (chunks * world * 4ull + 255ull) & ~255ull;
}

hipError_t launch_merge_export(const FlowSlot* table, const uint4* char_call, unsigned long long cap, uint32_t world,
                               uint32_t rank, unsigned long long shard_first, const unsigned long long* cmap,
                               fb_flow_mrec* out, unsigned long long out_cap, unsigned long long* d_counts,
                               void* scratch, hipStream_t s) {
    if (world == 0u || world > kMxMaxWorld) return hipErrorInvalidValue;
    const uint32_t chunks = (uint32_t)((cap + kMxChunk - 1) / kMxChunk);
    uint32_t* cnt = static_cast<uint32_t*>(scratch);
    hipLaunchKernelGGL(k_mx_count, dim3(chunks), dim3(64), 0, s, table, cap, world, cnt);
    hipLaunchKernelGGL(k_mx_scan, dim3(1), dim3(1024), 0, s, cnt, chunks, world, d_counts);
    hipLaunchKernelGGL(k_mx_write, dim3(chunks), dim3(64), 0, s, table, char_call, cap, world, rank, shard_first, cmap,
                       cnt, out, out_cap);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Record routing (fb_route_records_dev): a rank's dense SESSION records grouped by the owner of their
// key (stable: packet order inside a group), pkt_index made global (+ shard_first) and, with frame
// times, each record's capture time beside it.  The same count / scan / write structure as the
// export above, over records instead of table slots.
__device__ __forceinline__ uint32_t rec_owner(const fb_pkt_out* R, unsigned long long i, uint32_t world) {
    uint32_t key[10];
    __builtin_memcpy(key, &R[i].key, 40);
    key[9] &= 0xFFFFu;
    return flow_owner(flow_hash_words(key), world);
}

__global__ __launch_bounds__(64) void k_rt_count(const fb_pkt_out* R, const fb_batch_stats* st, uint32_t max_n,
                                                 uint32_t world, uint32_t* cnt) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long n = min((unsigned long long)st->n_session, (unsigned long long)max_n);
    const unsigned long long c0 = (unsigned long long)blockIdx.x * kMxChunk;
    uint32_t mine = 0u;
    for (uint32_t j = 0; j < kMxChunk; j += 64u) {
        const unsigned long long i = c0 + j + lane;
        const uint32_t o = i < n ? rec_owner(R, i, world) : ~0u;
        for (uint32_t w = 0; w < world; ++w) {
            const uint32_t k = (uint32_t)__popcll(__ballot(o == w));
            if (lane == w) mine += k;
        }
    }
    if (lane < world) cnt[(size_t)blockIdx.x * world + lane] = mine;
}

__global__ __launch_bounds__(64) void k_rt_write(const fb_pkt_out* R, const fb_batch_stats* st, uint32_t max_n,
                                                 uint32_t world, unsigned long long shard_first,
                                                 const unsigned long long* ts, const uint32_t* off, fb_pkt_out* out,
                                                 unsigned long long* ts_out) {
    const uint32_t lane = threadIdx.x;
    const unsigned long long n = min((unsigned long long)st->n_session, (unsigned long long)max_n);
    const unsigned long long c0 = (unsigned long long)blockIdx.x * kMxChunk;
    uint32_t next = lane < world ? off[(size_t)blockIdx.x * world + lane] : 0u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t j = 0; j < kMxChunk; j += 64u) {
        const unsigned long long i = c0 + j + lane;
        const bool in = i < n;
        const uint32_t o = in ? rec_owner(R, i, world) : ~0u;
        uint32_t pos = 0u;
        for (uint32_t w = 0; w < world; ++w) {
            const unsigned long long m = __ballot(o == w);
            const uint32_t base = (uint32_t)__shfl((int)next, (int)w, 64);
            if (o == w) pos = base + (uint32_t)__popcll(m & lt);
            if (lane == w) next += (uint32_t)__popcll(m);
        }
        if (in) {
            fb_pkt_out r = R[i];
            if (ts_out) ts_out[pos] = ts[r.pkt_index];
            r.pkt_index = (uint32_t)(r.pkt_index + shard_first);
            out[pos] = r;
        }
    }
}

uint64_t route_scratch_bytes(uint32_t max_n, uint32_t world) {
    const unsigned long long chunks = ((unsigned long long)max_n + kMxChunk - 1) / kMxChunk;
    return (std::max(chunks, 1ull) * world * 4ull + 255ull) & ~255ull;
}

hipError_t launch_route(const fb_pkt_out* recs, const fb_batch_stats* stats, uint32_t max_n, uint32_t world,
                        unsigned long long shard_first, const unsigned long long* ts, fb_pkt_out* out,
                        unsigned long long* ts_out, unsigned long long* d_counts, void* scratch, hipStream_t s) {
    if (world == 0u || world > kMxMaxWorld) return hipErrorInvalidValue;
    const uint32_t chunks = std::max<uint32_t>((uint32_t)(((unsigned long long)max_n + kMxChunk - 1) / kMxChunk), 1u);
    uint32_t* cnt = static_cast<uint32_t*>(scratch);
    hipLaunchKernelGGL(k_rt_count, dim3(chunks), dim3(64), 0, s, recs, stats, max_n, world, cnt);
    hipLaunchKernelGGL(k_mx_scan, dim3(1), dim3(1024), 0, s, cnt, chunks, world, d_counts);
    hipLaunchKernelGGL(k_rt_write, dim3(chunks), dim3(64), 0, s, recs, stats, max_n, world, shard_first, ts, cnt, out,
                       ts_out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Merge.  Scratch (per input record i unless noted): an open-addressing table of record indices
// (kMgLoad x n slots, power of two), head[i] = the record that claimed i's key, and per head the
// accumulators; rep[head] = the smallest index of the key's records (its output position).
struct MergeScratch {
    uint32_t* tab;                  // [tcap]
    uint32_t* head;                 // [n]
    uint32_t* rep;                  // [n] (per head) min record index
    unsigned long long* cnt;        // [n][6] counters
    unsigned long long* first;      // [n] min first_seen
    unsigned long long* last;       // [n] max last_seen
    unsigned long long* end;        // [n] min end_seen
    uint32_t* len;                  // [n] hist_len sum
    uint32_t* mask;                 // [n] hist_mask or
    uint32_t* emask;                // [n] end characters or
    uint32_t* r0;                   // [n] the ending rank
    uint32_t* seg;                  // [n] segment_count sum
    uint32_t* inseg;                // [n] in_segment of the latest packet's record
    uint32_t* sflags;               // [n] session_flags of the earliest packet's record
    uint32_t* blk;                  // [blocks + 1] output counts per block, then offsets
    unsigned long long tcap;
};
constexpr uint32_t kMgThreads = 256;

static unsigned long long merge_tcap(unsigned long long n) {
    unsigned long long t = 1024ull;
    while (t < 2ull * n) t <<= 1;
    return t;
}
static size_t al(size_t b) { return (b + 255) & ~size_t(255); }

uint64_t merge_scratch_bytes(unsigned long long n) {
    const unsigned long long blocks = (n + kMgThreads - 1) / kMgThreads;
    return al(merge_tcap(n) * 4) + 3 * al(n * 4) + al(n * 48) + 3 * al(n * 8) + 7 * al(n * 4) + al((blocks + 1) * 4);
}

static MergeScratch carve(void* base, unsigned long long n) {
    char* p = static_cast<char*>(base);
    MergeScratch m;
    m.tcap = merge_tcap(n);
    const unsigned long long blocks = (n + kMgThreads - 1) / kMgThreads;
    auto take = [&](size_t b) { char* q = p; p += al(b); return q; };
    m.tab = (uint32_t*)take(m.tcap * 4);
    m.head = (uint32_t*)take(n * 4);
    m.rep = (uint32_t*)take(n * 4);
    m.r0 = (uint32_t*)take(n * 4);
    m.cnt = (unsigned long long*)take(n * 48);
    m.first = (unsigned long long*)take(n * 8);
    m.last = (unsigned long long*)take(n * 8);
    m.end = (unsigned long long*)take(n * 8);
    m.len = (uint32_t*)take(n * 4);
    m.mask = (uint32_t*)take(n * 4);
    m.emask = (uint32_t*)take(n * 4);
    m.seg = (uint32_t*)take(n * 4);
    m.inseg = (uint32_t*)take(n * 4);
    m.sflags = (uint32_t*)take(n * 4);
    m.blk = (uint32_t*)take((blocks + 1) * 4);
    (void)take(0);
    return m;
}

__device__ __forceinline__ void key_of(const fb_flow_mrec& r, uint32_t k[10]) {
    __builtin_memcpy(k, &r.rec.key, 40);
    k[9] &= 0xFFFFu;
}

// Claim: each record finds the record that first claimed its key's table slot (linear probing).
__global__ __launch_bounds__(kMgThreads) void k_mg_claim(const fb_flow_mrec* in, unsigned long long n, MergeScratch m) {
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    if (i >= n) return;
    uint32_t k[10];
    key_of(in[i], k);
    unsigned long long t = flow_hash_words(k) & (m.tcap - 1ull);
    uint32_t hd = (uint32_t)i;
    for (unsigned long long probe = 0; probe < m.tcap; ++probe) {
        const uint32_t cur = atomicCAS(&m.tab[t], ~0u, (uint32_t)i);
        if (cur == ~0u) break;  // claimed: this record heads its key
        uint32_t o[10];
        key_of(in[cur], o);
        bool eq = true;
#pragma unroll
        for (int j = 0; j < 10; ++j) eq &= o[j] == k[j];
        if (eq) {
            hd = cur;
            break;
        }
        t = (t + 1ull) & (m.tcap - 1ull);
    }
    m.head[i] = hd;
    atomicMin(&m.rep[hd], (uint32_t)i);
}

// Order-independent reductions into the head's accumulators.
__global__ __launch_bounds__(kMgThreads) void k_mg_reduce(const fb_flow_mrec* in, unsigned long long n, MergeScratch m) {
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    if (i >= n) return;
    const fb_flow_rec& r = in[i].rec;
    const uint32_t hd = m.head[i];
    unsigned long long* c = m.cnt + (size_t)hd * 6u;
    atomicAdd(c + 0, (unsigned long long)r.outbound_bytes);
    atomicAdd(c + 1, (unsigned long long)r.inbound_bytes);
    atomicAdd(c + 2, (unsigned long long)r.orig_pkts);
    atomicAdd(c + 3, (unsigned long long)r.resp_pkts);
    atomicAdd(c + 4, (unsigned long long)r.orig_ip_bytes);
    atomicAdd(c + 5, (unsigned long long)r.resp_ip_bytes);
    atomicMin(m.first + hd, (unsigned long long)r.first_seen);
    atomicMax(m.last + hd, (unsigned long long)r.last_seen);
    if (r.end_seen != FB_SEEN_NONE) atomicMin(m.end + hd, (unsigned long long)r.end_seen);
    atomicAdd(m.len + hd, r.hist_len);
    atomicOr(m.mask + hd, (uint32_t)r.hist_mask);
    atomicAdd(m.seg + hd, r.segment_count);
}

// The ending rank: the record whose end is the key's smallest (positions are global, so exactly
// one); its end_mask is the character set of its own history at the end packet.
__global__ __launch_bounds__(kMgThreads) void k_mg_end(const fb_flow_mrec* in, unsigned long long n, MergeScratch m) {
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    if (i >= n) return;
    const fb_flow_rec& r = in[i].rec;
    const uint32_t hd = m.head[i];
    const unsigned long long E = m.end[hd];
    if (E != FB_SEEN_NONE && r.end_seen == E) {
        m.r0[hd] = r.slot;  // (the exporting rank)
        atomicOr(m.emask + hd, (uint32_t)r.end_mask);
    }
    // global positions are distinct per packet: exactly one record holds the key's latest packet
    // (in_segment follows it) and one its earliest (the insert, whose flags the session keeps)
    if (r.last_seen == m.last[hd]) m.inseg[hd] = r.in_segment;
    if (r.first_seen == m.first[hd]) m.sflags[hd] = r.session_flags;
}

// The other ranks' S s H h that precede the end packet: first occurrence in an earlier update
// call, or in the end's call on a lower rank.
__global__ __launch_bounds__(kMgThreads) void k_mg_before(const fb_flow_mrec* in, unsigned long long n,
                                                          MergeScratch m) {
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    if (i >= n) return;
    const fb_flow_mrec& x = in[i];
    const uint32_t hd = m.head[i];
    const unsigned long long E = m.end[hd];
    if (E == FB_SEEN_NONE || x.rec.end_seen == E) return;
    const uint32_t call_e = (uint32_t)(E >> 32), r0 = m.r0[hd], rank = x.rec.slot;
    uint32_t bits = 0u;
#pragma unroll
    for (uint32_t b = 0; b < 4u; ++b) {
        const uint32_t c = x.char_call[b];
        if (c != FB_CALL_NONE && (c < call_e || (c == call_e && rank < r0))) bits |= 1u << b;
    }
    if (bits) atomicOr(m.emask + hd, bits);
}

// Output positions: each key's record goes where its first input record is in the order of first
// records (block counts, one scan, then the block's ballot prefix).
__global__ __launch_bounds__(kMgThreads) void k_mg_count(unsigned long long n, MergeScratch m) {
    __shared__ uint32_t ws[kMgThreads / 64];
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    const bool f = i < n && m.rep[m.head[i]] == (uint32_t)i;
    const uint32_t c = (uint32_t)__popcll(__ballot(f));
    if ((threadIdx.x & 63u) == 0u) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0u;
        for (uint32_t w = 0; w < kMgThreads / 64u; ++w) t += ws[w];
        m.blk[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(1024) void k_mg_scan(MergeScratch m, uint32_t blocks, unsigned long long* d_n) {
    __shared__ uint32_t ws[16];
    // each thread scans a contiguous run of block counts
    const uint32_t per = (blocks + 1023u) / 1024u, b0 = threadIdx.x * per, b1 = min(b0 + per, blocks);
    uint32_t s = 0u;
    for (uint32_t b = b0; b < b1; ++b) s += m.blk[b];
    uint32_t tot;
    uint32_t run = wg_excl_scan(s, ws, tot);
    if (threadIdx.x == 0) *d_n = tot;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t v = m.blk[b];
        m.blk[b] = run;
        run += v;
    }
}
__global__ __launch_bounds__(kMgThreads) void k_mg_write(const fb_flow_mrec* in, unsigned long long n, MergeScratch m,
                                                         fb_flow_rec* out) {
    __shared__ uint32_t ws[kMgThreads / 64];
    const unsigned long long i = (unsigned long long)blockIdx.x * kMgThreads + threadIdx.x;
    const uint32_t hd = i < n ? m.head[i] : 0u;
    const bool f = i < n && m.rep[hd] == (uint32_t)i;
    const unsigned long long b = __ballot(f);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0u) ws[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    if (!f) return;
    uint32_t pos = m.blk[blockIdx.x] + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    for (uint32_t w = 0; w < wave; ++w) pos += ws[w];
    const fb_flow_rec& r = in[i].rec;
    fb_flow_rec o;
    o.key = r.key;
    const unsigned long long* c = m.cnt + (size_t)hd * 6u;
    o.outbound_bytes = c[0];
    o.inbound_bytes = c[1];
    o.orig_pkts = c[2];
    o.resp_pkts = c[3];
    o.orig_ip_bytes = c[4];
    o.resp_ip_bytes = c[5];
    o.first_seen = m.first[hd];
    o.last_seen = m.last[hd];
    const unsigned long long E = m.end[hd];
    o.end_seen = E;  // FB_SEEN_NONE when no rank saw a FIN/RST
    o.hist_len = m.len[hd];
    o.hist_mask = (uint16_t)m.mask[hd];
    const uint32_t em = E != FB_SEEN_NONE ? (m.emask[hd] & 0xFFu) : 0u;
    o.conn_state = (uint8_t)(E != FB_SEEN_NONE ? conn_state_of(em) : FB_CONN_NONE);
    o.end_mask = (uint8_t)em;
    o.slot = 0u;
    o.session_flags = m.sflags[hd];
    o.segment_count = m.seg[hd];
    o.in_segment = (uint8_t)m.inseg[hd];
    o.reserved[0] = o.reserved[1] = o.reserved[2] = 0u;
    out[pos] = o;
}

hipError_t launch_merge(const fb_flow_mrec* in, unsigned long long n, fb_flow_rec* out, unsigned long long* d_n,
                        void* scratch, hipStream_t s) {
    if (n == 0ull) return hipMemsetAsync(d_n, 0, 8, s);
    if (n >= 0xFFFFFFFFull) return hipErrorInvalidValue;
    const MergeScratch m = carve(scratch, n);
    const uint32_t blocks = (uint32_t)((n + kMgThreads - 1) / kMgThreads);
    hipError_t e;
    if ((e = hipMemsetAsync(m.tab, 0xFF, m.tcap * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.rep, 0xFF, n * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.cnt, 0, n * 48, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.first, 0xFF, n * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.last, 0, n * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.end, 0xFF, n * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.len, 0, n * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.mask, 0, n * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.emask, 0, n * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(m.seg, 0, n * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_mg_claim, dim3(blocks), dim3(kMgThreads), 0, s, in, n, m);
    hipLaunchKernelGGL(k_mg_reduce, dim3(blocks), dim3(kMgThreads), 0, s, in, n, m);
    hipLaunchKernelGGL(k_mg_end, dim3(blocks), dim3(kMgThreads), 0, s, in, n, m);
    hipLaunchKernelGGL(k_mg_before, dim3(blocks), dim3(kMgThreads), 0, s, in, n, m);
    hipLaunchKernelGGL(k_mg_count, dim3(blocks), dim3(kMgThreads), 0, s, n, m);
    hipLaunchKernelGGL(k_mg_scan, dim3(1), dim3(1024), 0, s, m, blocks, d_n);
    hipLaunchKernelGGL(k_mg_write, dim3(blocks), dim3(kMgThreads), 0, s, in, n, m, out);
    return hipGetLastError();
}

}  // namespace fbk

extern "C" uint32_t fb_flow_owner(const fb_session_key* key, uint32_t world) {
    uint32_t w[10];
    __builtin_memcpy(w, key, 40);
    w[9] &= 0xFFFFu;
    return world ? fbk::flow_owner(fbk::flow_hash_words(w), world) : 0u;
}
