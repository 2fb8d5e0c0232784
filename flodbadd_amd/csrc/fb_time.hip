// fb_time.hip -- capture-time state of the session table (timed contexts, FB_CFG_TIMED).
//
// The reference stamps every packet with the wall clock (`now = Utc::now()`, src/packets.rs:230)
// and keeps per session start_time / last_activity / end_time and the segment state
// (update_session_stats, src/packets.rs:137-200; insert 352-380, 414-426): a TCP packet with PSH
// ends the open segment, and so does any packet arriving >= 5 s (segment_timeout) after the flow's
// previous one, which then opens a new segment at itself; each ended segment after the first adds
// the gap between its start and the previous segment's end to the interarrival sum.  On a timed
// context every update call carries the frames' capture timestamps, and this pass -- after the
// update's K2 has placed every record's flow in the table -- brings each touched flow's time record
// (FlowTime, one per table slot: the "time plane") forward over the batch's packets of that flow in
// packet order.
//
// The state machine looks sequential, but it is local to consecutive packets of a flow.  With T_i
// = (the gap to the flow's previous packet, in chrono's truncated ms) >= 5000 and P_i = TCP with PSH:
//   in_i    = T_i || !P_i          (in_segment after packet i; the insert packet: !P_0)
//   end_i   = P_i || (in_{i-1} && T_i)    (a segment ends at i; the insert: P_0)
//   reset_i = T_i || !in_{i-1}     (current_segment_start := t_i; the insert: always)
// and at an end the interarrival term is (segment start as of i) - (previous end), where the start
// is t_i when !in_{i-1} (the segment opened at i) and otherwise the start current before i.  So one
// stable sort of the batch's records by table slot (they arrive in packet order) makes each flow's
// packets one contiguous run, and two chained segmented scans over the runs give every packet its
// inputs -- scan A: the latest reset / end in the run at or before it, the run's ends so far, its
// head; scan B: the accepted interarrival sum and the latest accepted term with its divisor -- and
// the run's last packet writes the flow's new FlowTime:
//   K2           writes the sort input at each applied record's slot (FlowParams::tkv): table slot
//                << 32 | pkt_index << 1 | P; record slots without an entry keep launch_time_prepare's
//                "no flow" word (~0: sorts last).  K1c's combining is off on a timed context, so every
//                record is a plain entry
//   sort         rocPRIM onesweep LSD radix sort of (slot << 1 | P, capture time) pairs on the slot bits
//                (stable: the packet order inside a slot stays), its inputs read from K2's words
//                through transform iterators -- the time is ts[pkt_index], so the sort also gathers
//                the times into sorted order (record slots follow packet order: a near-sequential read)
//   k_time_runs  ONE launch over tiles of 2,048 sorted packets taken in ticket order: per packet its
//                time, T / in / end / reset (its predecessor's `in` from the packet before that),
//                scan A (thread, wave, block, then the tile's prefix by decoupled look-back), the
//                interarrival term, scan B the same way, and the runs' last packets write the plane
//                (start / end from the table's positions of this call)
// Bytes per record: K2's 8-B sort input store (one per record, at its record slot); the sort's
// histogram 8 B, its first pass 8 + 8 in (word, time) and 12 out, its second 12 + 12; the fused pass
// 12 B in + the timestamp reads (8 B, up to four per packet, mostly cached) -- an auxiliary pass, not
// the headline path.  The insert test needs no pkt_index: a flow whose first_seen is of this batch was
// inserted by this call, at its run's head.
#include <cstring>  // (rocPRIM's texture-cache iterator needs memset declared)

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "fb_internal.h"

namespace fbk {

namespace {

constexpr uint32_t kTmThreads = 256;

// chrono's (a - b).num_milliseconds(): the signed difference truncated toward zero
__device__ __forceinline__ long long ms_between(unsigned long long a, unsigned long long b) {
    return ((long long)a - (long long)b) / 1000000ll;
}
__device__ __forceinline__ bool timeout_of(unsigned long long now, unsigned long long last) {
    return ms_between(now, last) >= (long long)FB_SEGMENT_TIMEOUT_MS;
}

// Segmented scan words of the fused pass (k_time_runs): values since the latest run head at or before
// an element, so nothing needs the run's head position to discount earlier runs.
//   SegA: head index + 1 (0: no head in the segment) | the run is a new flow's (bit 31); the latest
//         reset / end (index + 1, 0: none in the run); the run's ends so far
//   SegB: the run's accepted interarrival ms so far; the latest accepted term (index + 1); its
//         divisor | head bit 30
struct SegA {
    uint32_t h, r, e, c;
};
struct SegB {
    long long s;
    uint32_t a, d;
};
constexpr uint32_t kInsRun = 0x80000000u;
__device__ __forceinline__ bool segA_head(const SegA& x) { return (x.h & ~kInsRun) != 0u; }
__device__ __forceinline__ SegA segA_op(const SegA& x, const SegA& y) {
    if (segA_head(y)) return y;
    return SegA{x.h, x.r > y.r ? x.r : y.r, x.e > y.e ? x.e : y.e, x.c + y.c};
}
// SegB's head flag rides in bit 30 of d (a is 0 for a segment without a term)
constexpr uint32_t kBHead = 0x40000000u;
__device__ __forceinline__ SegB segB_op(const SegB& x, const SegB& y) {
    if (y.d & kBHead) return y;
    SegB o;
    o.s = x.s + y.s;
    const bool take_y = y.a > x.a;
    o.a = take_y ? y.a : x.a;
    o.d = ((take_y ? y.d : x.d) & ~kBHead) | (x.d & kBHead);
    return o;
}

// per sorted packet flags
constexpr uint8_t kFP = 1u, kFT = 2u, kFIn = 4u, kFHead = 8u, kFIns = 16u, kFEnd = 32u, kFInPrev = 64u, kFReset = 128u;

}  // namespace

// ---------------------------------------------------------------------------------------------
// The fused pass over the sorted packets (one launch, tiles of kRunTile packets taken in ticket order,
// two chained decoupled look-backs): per packet its flags, the segmented scan A (latest reset / end,
// ends so far, the run's head), then its interarrival term and the segmented scan B (accepted sum,
// latest accepted term and its divisor), and the run's last packet writes the flow's FlowTime.
//
// A tile publishes each scan's aggregate, then its inclusive value, as two 64-bit words with RELAXED
// agent-scope atomic stores, each word carrying a 2-bit status (1 aggregate, 2 inclusive) beside its
// half of the value: a reader takes a value only when both of its words carry the status, so no
// release / acquire fence is needed (on gfx950 an agent-scope release writes back, and an acquire
// invalidates, the XCD's L2 -- per tile, that made this pass ~8x slower than its memory traffic).
constexpr uint32_t kRunThreads = 512, kRunItems = 4, kRunTile = kRunThreads * kRunItems;
constexpr unsigned long long kStAgg = 1ull, kStInc = 2ull;

struct RunStatus {  // per tile 8 words: A aggregate, A inclusive, B aggregate, B inclusive (zeroed per launch)
    unsigned long long* w;
    uint32_t* ticket;
};
constexpr unsigned long long kM27 = (1ull << 27) - 1ull, kM28 = (1ull << 28) - 1ull;
__device__ __forceinline__ void pack(const SegA& x, unsigned long long st, unsigned long long (&w)[2]) {
    w[0] = st | (unsigned long long)x.h << 2 | ((unsigned long long)x.r & kM27) << 34;  // h: 27 bits + bit 31
    w[1] = st | ((unsigned long long)x.e & kM27) << 2 | ((unsigned long long)x.c & kM27) << 29;
}
__device__ __forceinline__ SegA unpack_a(const unsigned long long (&w)[2]) {
    return SegA{(uint32_t)(w[0] >> 2), (uint32_t)((w[0] >> 34) & kM27), (uint32_t)((w[1] >> 2) & kM27),
                (uint32_t)((w[1] >> 29) & kM27)};
}
constexpr unsigned long long kM46 = (1ull << 46) - 1ull;
__device__ __forceinline__ void pack(const SegB& x, unsigned long long st, unsigned long long (&w)[2]) {
    // s: 46 bits (accepted interarrivals are >= 0), a: 27 bits, d: 28 bits (divisor + head bit 30 -> 27)
    const unsigned long long d = (x.d & kM27) | ((x.d & kBHead) ? (1ull << 27) : 0ull);
    w[0] = st | ((unsigned long long)x.s & kM46) << 2 | ((unsigned long long)x.a & 0xFFFFull) << 48;
    w[1] = st | (((unsigned long long)x.a >> 16) & 0x7FFull) << 2 | (d & kM28) << 13;
}
__device__ __forceinline__ SegB unpack_b(const unsigned long long (&w)[2]) {
    const uint32_t d = (uint32_t)((w[1] >> 13) & kM28);
    return SegB{(long long)((w[0] >> 2) & kM46), (uint32_t)((w[0] >> 48) | ((w[1] >> 2) & 0x7FFull) << 16),
                (d & (uint32_t)kM27) | ((d >> 27) ? kBHead : 0u)};
}
__device__ __forceinline__ void st_put(unsigned long long* p, const unsigned long long (&w)[2]) {
    __hip_atomic_store(p, w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool st_get(const unsigned long long* p, unsigned long long st, unsigned long long (&w)[2]) {
    w[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w[1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (w[0] & 3ull) == st && (w[1] & 3ull) == st;
}
__device__ __forceinline__ bool has_head(const SegA& x) { return segA_head(x); }
__device__ __forceinline__ bool has_head(const SegB& x) { return (x.d & kBHead) != 0u; }
__device__ __forceinline__ SegA unpack(const unsigned long long (&w)[2], const SegA*) { return unpack_a(w); }
__device__ __forceinline__ SegB unpack(const unsigned long long (&w)[2], const SegB*) { return unpack_b(w); }

// Lane shuffles of the scan words.
__device__ __forceinline__ SegA shfl_down(const SegA& x, int o) {
    return SegA{(uint32_t)__shfl_down(x.h, o, 64), (uint32_t)__shfl_down(x.r, o, 64), (uint32_t)__shfl_down(x.e, o, 64),
                (uint32_t)__shfl_down(x.c, o, 64)};
}
__device__ __forceinline__ SegB shfl_down(const SegB& x, int o) {
    return SegB{__shfl_down(x.s, o, 64), (uint32_t)__shfl_down(x.a, o, 64), (uint32_t)__shfl_down(x.d, o, 64)};
}

// The exclusive prefix of tile `t` for one scan (words at offset `off` of each tile's 8: 0 A, 4 B), by
// one wavefront: lane L looks at tile t-1-L-64k (lane 0 the nearest); the walk ends at the nearest
// tile whose inclusive value is published or whose aggregate holds a run head (a segmented value),
// waiting only for that tile and the nearer ones; the window is folded in tile order (the all-zero
// word is the identity of both operators).
template <class V, class Op>
__device__ V lookback(const RunStatus& S, uint32_t t, uint32_t off, Op op) {
    const uint32_t lane = threadIdx.x & 63u;
    V acc{};
    bool have = false;
    for (int j0 = (int)t - 1; j0 >= 0; j0 -= 64) {
        const int j = j0 - (int)lane;
        bool ready = j < 0, inc = false;
        V v{};
        uint32_t stop;
        for (;;) {
            if (!ready) {
                unsigned long long w[2];
                const unsigned long long* base = S.w + (size_t)j * 8u + off;
                if (st_get(base + 2, kStInc, w)) {
                    v = unpack(w, (const V*)nullptr);
                    ready = inc = true;
                } else if (st_get(base, kStAgg, w)) {
                    v = unpack(w, (const V*)nullptr);
                    ready = true;
                }
            }
            const unsigned long long rdy = __ballot(ready);
            const unsigned long long hit = __ballot(ready && j >= 0 && (inc || has_head(v)));
            const uint32_t not_ready = ~rdy ? (uint32_t)__builtin_ctzll(~rdy) : 64u;
            const uint32_t first_hit = hit ? (uint32_t)__builtin_ctzll(hit) : 64u;
            if (first_hit < not_ready || not_ready == 64u) {
                stop = first_hit;  // (64: the whole window, no end of the walk in it)
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (j < 0 || lane > stop) v = V{};
        // fold: lane L holds tiles [L, L + o) after step o (higher lanes are earlier tiles)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const V w = shfl_down(v, o);
            if ((lane & (2u * o - 1u)) == 0u) v = op(w, v);
        }
        acc = have ? op(v, acc) : v;  // (lane 0 holds the window folded in tile order)
        have = true;
        if (stop < 64u) break;
    }
    return acc;  // meaningful in lane 0
}

// The capture time of sorted packet j: the sort carried it beside the key (its value), so the fused
// pass reads it coalesced (a packet reads its own and its two predecessors').
__device__ __forceinline__ unsigned long long t_of(const unsigned long long* tsort, uint32_t j) { return tsort[j]; }

// The sort's inputs, read straight from K2's words through rocPRIM transform iterators (no pass of
// their own): the key table slot << 1 | P (a "no flow" word's slot ~0u gives 0x7FFFFFFF, past every
// slot: it sorts last), the value the record's capture time ts[pkt_index] (record slots follow packet
// order, so these reads walk the timestamp array nearly in order).
struct TimeSortKey {
    __host__ __device__ uint32_t operator()(unsigned long long w) const {
        return (uint32_t)(w >> 32) << 1 | ((uint32_t)w & 1u);
    }
};
struct TimeSortTs {
    const unsigned long long* ts;
    uint32_t cap;
    __host__ __device__ unsigned long long operator()(unsigned long long w) const {
        return (uint32_t)(w >> 32) < cap ? ts[(uint32_t)w >> 1] : 0ull;
    }
};

// the sorted keys: table slot (>= cap: no flow) << 1 | P
#define TKEY(i) (ks[(i)] >> 1)
#define TPSH(i) (ks[(i)] & 1u)

__global__ __launch_bounds__(kRunThreads) void k_time_runs(const uint32_t* ks, uint32_t n,
                                                          uint32_t cap, const FlowSlot* T, FlowTime* plane,
                                                          const unsigned long long* ts, const unsigned long long* tsort,
                                                          uint32_t batch, RunStatus S) {
    __shared__ uint32_t s_tile;
    __shared__ SegA s_wa[kRunThreads / 64];
    __shared__ SegB s_wb[kRunThreads / 64];
    __shared__ SegA s_pa;
    __shared__ SegB s_pb;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(S.ticket, 1u);  // tiles in start order: the look-back waits only on running ones
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * kRunTile + tid * kRunItems;

    // Per packet i: its T / in / insert and its predecessor's `in` (from the packet before that, or the
    // plane at a run head).  The loads go out together first -- key words, times and, for a packet at
    // run position 0 or 1, the slot's first_seen and plane words, none behind another -- then the flags
    // are computed (a timing-only split of this pass put ~35 % of it in the plane / table round trips).
    uint32_t key[kRunItems];
    uint8_t fl[kRunItems];
    unsigned long long tt[kRunItems];
    SegA xa[kRunItems];
    unsigned long long tp[kRunItems], tpp[kRunItems], fs[kRunItems], la[kRunItems];
    uint8_t vv[kRunItems], vp[kRunItems];  // P of the packet and of its predecessor
    uint8_t pos[kRunItems], isg[kRunItems];  // run position: 0 head, 1 after the head, 2 later
#pragma unroll
    for (uint32_t k = 0; k < kRunItems; ++k) {
        const uint32_t i = base + k;
        key[k] = i < n ? TKEY(i) : cap;
        const uint32_t s = key[k];
        const bool ok = s < cap;
        const bool head = ok && (i == 0u || TKEY(i - 1u) != s);
        const bool head1 = ok && !head && (i == 1u || TKEY(i - 2u) != s);
        pos[k] = head ? 0u : head1 ? 1u : 2u;
        tt[k] = ok ? t_of(tsort, i) : 0ull;
        vv[k] = ok ? TPSH(i) : 0u;
        tp[k] = ok && !head ? t_of(tsort, i - 1u) : 0ull;
        vp[k] = ok && !head ? TPSH(i - 1u) : 0u;
        tpp[k] = ok && !head && !head1 ? t_of(tsort, i - 2u) : 0ull;
        const bool need = ok && (head || head1);
        fs[k] = need ? T[s].first_seen : FB_SEEN_NONE;
        la[k] = need ? plane[s].last_activity_ns : 0ull;
        isg[k] = need ? plane[s].in_segment : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kRunItems; ++k) {
        const uint32_t i = base + k;
        fl[k] = 0u;
        xa[k] = SegA{0u, 0u, 0u, 0u};
        if (key[k] >= cap) continue;  // (no flow: sorts last, a neutral word)
        const bool head = pos[k] == 0u;
        const unsigned long long t = tt[k];
        const bool P_ = vv[k] & 1u;
        bool Ti, ini, insi, in_prev;
        // The flow was inserted by this call exactly when its first_seen is of this batch (the update
        // keeps a new flow's first_seen at its earliest packet), and then its insert packet is the
        // run's head: the run holds every applied packet of the flow, in packet order.
        const bool new_flow = (fs[k] >> 32) == (unsigned long long)batch;
        if (head) {
            insi = new_flow;  // the flow's insert is this packet
            Ti = !insi && timeout_of(t, la[k]);
            ini = insi ? !P_ : (Ti || !P_);
            in_prev = insi ? false : isg[k] != 0u;
        } else {
            insi = false;
            Ti = timeout_of(t, tp[k]);
            ini = Ti || !P_;
            const bool P1 = vp[k] & 1u;
            if (pos[k] == 1u) {  // the predecessor is the run's head
                const bool ins1 = new_flow;  // (the head inserted the flow)
                const bool T1 = !ins1 && timeout_of(tp[k], la[k]);
                in_prev = ins1 ? !P1 : (T1 || !P1);
            } else {
                const bool T1 = timeout_of(tp[k], tpp[k]);
                in_prev = T1 || !P1;
            }
        }
        const bool end = insi ? P_ : (P_ || (in_prev && Ti));
        const bool reset = insi || Ti || !in_prev;
        fl[k] = (uint8_t)((P_ ? kFP : 0u) | (Ti ? kFT : 0u) | (ini ? kFIn : 0u) | (head ? kFHead : 0u) |
                          (insi ? kFIns : 0u) | (end ? kFEnd : 0u) | (in_prev ? kFInPrev : 0u) | (reset ? kFReset : 0u));
        xa[k] = SegA{head ? ((i + 1u) | (insi ? kInsRun : 0u)) : 0u, reset ? i + 1u : 0u, end ? i + 1u : 0u,
                     end ? 1u : 0u};
    }
    // ---- scan A: thread-sequential, wave, block, then the tile's prefix by look-back
    SegA ia[kRunItems];  // inclusive within the thread's items
    ia[0] = xa[0];
#pragma unroll
    for (uint32_t k = 1; k < kRunItems; ++k) ia[k] = segA_op(ia[k - 1], xa[k]);
    SegA tot = ia[kRunItems - 1];
    SegA wincl = tot;  // wave inclusive scan of the thread totals
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        SegA y;
        y.h = __shfl_up(wincl.h, o, 64);
        y.r = __shfl_up(wincl.r, o, 64);
        y.e = __shfl_up(wincl.e, o, 64);
        y.c = __shfl_up(wincl.c, o, 64);
        if (lane >= (uint32_t)o) wincl = segA_op(y, wincl);
    }
    if (lane == 63u) s_wa[wave] = wincl;
    SegA wexcl;  // exclusive within the wave
    wexcl.h = __shfl_up(wincl.h, 1, 64);
    wexcl.r = __shfl_up(wincl.r, 1, 64);
    wexcl.e = __shfl_up(wincl.e, 1, 64);
    wexcl.c = __shfl_up(wincl.c, 1, 64);
    __syncthreads();
    if (wave == 0u) {
        SegA agg = s_wa[0];
        for (uint32_t w = 1; w < kRunThreads / 64; ++w) agg = segA_op(agg, s_wa[w]);
        SegA prefix{0u, 0u, 0u, 0u};
        unsigned long long pw[2];
        if (tile == 0u) {
            if (lane == 0u) {
                pack(agg, kStInc, pw);
                st_put(S.w + 2, pw);
            }
        } else {
            if (lane == 0u) {
                pack(agg, kStAgg, pw);
                st_put(S.w + (size_t)tile * 8u, pw);
            }
            prefix = lookback<SegA>(S, tile, 0u, segA_op);
            if (lane == 0u) {
                pack(segA_op(prefix, agg), kStInc, pw);
                st_put(S.w + (size_t)tile * 8u + 2u, pw);
            }
        }
        if (lane == 0u) s_pa = prefix;
    }
    __syncthreads();
    {
        SegA pre = s_pa;  // everything before this thread's first item
        for (uint32_t w = 0; w < wave; ++w) pre = segA_op(pre, s_wa[w]);
        if (lane > 0u) pre = segA_op(pre, wexcl);
        SegA ex[kRunItems];  // exclusive per item (= inclusive of the element before)
        ex[0] = pre;
#pragma unroll
        for (uint32_t k = 1; k < kRunItems; ++k) ex[k] = segA_op(pre, ia[k - 1]);
#pragma unroll
        for (uint32_t k = 0; k < kRunItems; ++k) {
            ia[k] = segA_op(pre, ia[k]);  // inclusive, global
            xa[k] = ex[k];
        }
    }
    // ---- interarrival terms and scan B
    SegB xb[kRunItems];
#pragma unroll
    for (uint32_t k = 0; k < kRunItems; ++k) {
        const uint32_t i = base + k;
        xb[k] = SegB{0ll, 0u, (fl[k] & kFHead) ? kBHead : 0u};
        if (key[k] >= cap || !(fl[k] & kFEnd) || (fl[k] & kFIns)) continue;
        const uint32_t s = key[k];
        const SegA& inc = ia[k];
        const bool ins_run = inc.h & kInsRun;
        const bool head = fl[k] & kFHead;
        const SegA prev = head ? SegA{0u, 0u, 0u, 0u} : xa[k];  // the run's state before packet i
        unsigned long long prev_end = FB_SEEN_NONE;
        if (prev.e) prev_end = t_of(tsort, prev.e - 1u);
        else if (!ins_run) prev_end = plane[s].last_segment_end_ns;
        if (prev_end == FB_SEEN_NONE) continue;
        unsigned long long start;  // current_segment_start as of packet i (src/packets.rs:151-154)
        if (!(fl[k] & kFInPrev)) start = tt[k];
        else if (prev.r) start = t_of(tsort, prev.r - 1u);
        else start = plane[s].current_segment_start_ns;
        const long long ia_ms = ms_between(start, prev_end);
        if (ia_ms < 0) continue;  // (double)ia / 1000.0 >= 0.0, src/packets.rs:165
        const uint32_t before = prev.c + (ins_run ? 0u : plane[s].segment_count);
        xb[k] = SegB{ia_ms, i + 1u, before | (head ? kBHead : 0u)};
    }
    SegB ib[kRunItems];
    ib[0] = xb[0];
#pragma unroll
    for (uint32_t k = 1; k < kRunItems; ++k) ib[k] = segB_op(ib[k - 1], xb[k]);
    SegB wb = ib[kRunItems - 1];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        SegB y;
        y.s = __shfl_up(wb.s, o, 64);
        y.a = __shfl_up(wb.a, o, 64);
        y.d = __shfl_up(wb.d, o, 64);
        if (lane >= (uint32_t)o) wb = segB_op(y, wb);
    }
    if (lane == 63u) s_wb[wave] = wb;
    SegB wbx;
    wbx.s = __shfl_up(wb.s, 1, 64);
    wbx.a = __shfl_up(wb.a, 1, 64);
    wbx.d = __shfl_up(wb.d, 1, 64);
    __syncthreads();
    if (wave == 0u) {
        SegB agg = s_wb[0];
        for (uint32_t w = 1; w < kRunThreads / 64; ++w) agg = segB_op(agg, s_wb[w]);
        SegB prefix{0ll, 0u, 0u};
        unsigned long long pw[2];
        if (tile == 0u) {
            if (lane == 0u) {
                pack(agg, kStInc, pw);
                st_put(S.w + 6, pw);
            }
        } else {
            if (lane == 0u) {
                pack(agg, kStAgg, pw);
                st_put(S.w + (size_t)tile * 8u + 4u, pw);
            }
            prefix = lookback<SegB>(S, tile, 4u, segB_op);
            if (lane == 0u) {
                pack(segB_op(prefix, agg), kStInc, pw);
                st_put(S.w + (size_t)tile * 8u + 6u, pw);
            }
        }
        if (lane == 0u) s_pb = prefix;
    }
    __syncthreads();
    SegB preb = s_pb;
    for (uint32_t w = 0; w < wave; ++w) preb = segB_op(preb, s_wb[w]);
    if (lane > 0u) preb = segB_op(preb, wbx);
    // ---- each run's last packet: the flow's new time record
#pragma unroll
    for (uint32_t k = 0; k < kRunItems; ++k) {
        const uint32_t i = base + k;
        const uint32_t s = key[k];
        if (s >= cap || (i + 1u < n && TKEY(i + 1u) == s)) continue;
        const SegA a = ia[k];
        const SegB b = segB_op(preb, ib[k]);
        const uint32_t H = (a.h & ~kInsRun) - 1u;
        const bool ins = a.h & kInsRun;
        FlowTime o;
        if (ins) {
            o.start_time_ns = t_of(tsort, H);
            o.end_time_ns = FB_SEEN_NONE;
            o.current_segment_start_ns = o.start_time_ns;
            o.last_segment_end_ns = FB_SEEN_NONE;
            o.total_segment_interarrival_ms = 0ll;
            o.segment_interarrival_div = 0u;
            o.segment_count = 0u;
        } else {
            o = plane[s];
        }
        o.segment_count += a.c;
        if (a.r) o.current_segment_start_ns = t_of(tsort, a.r - 1u);
        if (a.e) o.last_segment_end_ns = t_of(tsort, a.e - 1u);
        o.total_segment_interarrival_ms += b.s;
        if (b.a) o.segment_interarrival_div = b.d & ~kBHead;
        o.last_activity_ns = tt[k];
        o.in_segment = (fl[k] & kFIn) ? 1u : 0u;
        // end_time at the flow's first FIN/RST, which the update placed in end_seen (src/packets.rs:195-198)
        const unsigned long long es = T[s].end_seen;
        if (es != FB_SEEN_NONE && (es >> 32) == (unsigned long long)batch && o.end_time_ns == FB_SEEN_NONE)
            o.end_time_ns = ts[es & 0xFFFFFFFFull];
        o.reserved[0] = o.reserved[1] = o.reserved[2] = 0u;
        o.slot = 0u;
        plane[s] = o;
    }
}

// Growth: the time records follow their flows (remap[old slot] = new slot, ~0u: empty).
__global__ __launch_bounds__(kTmThreads) void k_time_remap(const FlowTime* old, const uint32_t* remap,
                                                           unsigned long long old_cap, FlowTime* nw) {
    const unsigned long long i = (unsigned long long)blockIdx.x * kTmThreads + threadIdx.x;
    if (i >= old_cap) return;
    const uint32_t d = remap[i];
    if (d != ~0u) nw[d] = old[i];
}

// fb_flow_export_times_dev: every flow's time record with its slot.
__global__ __launch_bounds__(256) void k_time_export(const FlowSlot* T, const FlowTime* plane, unsigned long long cap,
                                                     fb_flow_time* out, unsigned long long out_cap,
                                                     unsigned long long* d_n) {
    __shared__ unsigned long long sh[4];
    __shared__ unsigned long long s_base;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < cap; base += stride) {
        const unsigned long long i = base + threadIdx.x;
        const bool occ = i < cap && T[i].tag >= 2u;
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
            fb_flow_time o = plane[i];
            o.slot = (uint32_t)i;
            out[pos] = o;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// The sort: rocPRIM's onesweep LSD radix sort of (key, time) pairs on the key's slot bits [1, 2 +
// log2(cap)), FB_TIME_RADIX_BITS per pass (11: a 2^21-slot table's 22 bits in two passes instead of
// three at rocPRIM's default 8), tiles of 1024 x 16 pairs (2,048 digits need the larger tiles: 8
// items per thread 1,819 us per timed 10.5M-frame C4 call, 12 1,779, 16 1,740, 20 1,757, 24 1,802,
// 32 1,967; 8-bit digits 1,851, 10-bit 1,849; profiles/r06_timed_sort_pairs_ab.txt).
#ifndef FB_TIME_RADIX_BITS
#define FB_TIME_RADIX_BITS 11
#endif
#ifndef FB_TIME_SORT_BLOCK
#define FB_TIME_SORT_BLOCK 1024
#endif
#ifndef FB_TIME_SORT_ITEMS
#define FB_TIME_SORT_ITEMS 16
#endif
using TimeSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<FB_TIME_SORT_BLOCK, FB_TIME_SORT_ITEMS>,
                                        rocprim::kernel_config<FB_TIME_SORT_BLOCK, FB_TIME_SORT_ITEMS>,
                                        FB_TIME_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;
using TimeKeyIt = rocprim::transform_iterator<const unsigned long long*, TimeSortKey, uint32_t>;
using TimeTsIt = rocprim::transform_iterator<const unsigned long long*, TimeSortTs, unsigned long long>;

static hipError_t time_sort(void* tmp, size_t& tmp_bytes, const unsigned long long* kv, uint32_t* ks,
                            unsigned long long* tsort, const unsigned long long* ts, uint32_t cap, uint32_t n,
                            uint32_t bits, hipStream_t st) {
    return rocprim::radix_sort_pairs<TimeSortConfig>(tmp, tmp_bytes, TimeKeyIt(kv, TimeSortKey{}), ks,
                                                     TimeTsIt(kv, TimeSortTs{ts, cap}), tsort, n, 1u, 1u + bits, st);
}

struct TimeScratch {
    unsigned long long* kv;
    uint32_t* ks;
    unsigned long long* tsort;
    RunStatus st;
    uint32_t tiles;
    void* tmp;
    size_t tmp_bytes;
};
static size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

static size_t sort_tmp_bytes(uint32_t n, uint32_t bits) {
    size_t a = 0;
    if (time_sort(nullptr, a, nullptr, nullptr, nullptr, nullptr, 0u, n, bits, (hipStream_t)0) != hipSuccess)
        a = 0;  // (the sort itself then reports the error)
    return a;
}

uint64_t time_scratch_bytes(uint32_t n, uint32_t cap_bits) {
    const size_t m = std::max<uint32_t>(n, 1u);
    const size_t tiles = (m + kRunTile - 1) / kRunTile;
    return al256(m * 8) * 2 + al256(m * 4) + al256(tiles * 64) + al256(8) + al256(sort_tmp_bytes(n, cap_bits + 1u));
}

static TimeScratch carve(void* base, uint32_t n, uint32_t cap_bits) {
    char* p = static_cast<char*>(base);
    const size_t m = std::max<uint32_t>(n, 1u);
    auto take = [&](size_t b) { char* q = p; p += al256(b); return q; };
    TimeScratch s;
    s.tiles = (uint32_t)((m + kRunTile - 1) / kRunTile);
    s.kv = (unsigned long long*)take(m * 8);  // (first: time_key_array)
    s.ks = (uint32_t*)take(m * 4);
    s.tsort = (unsigned long long*)take(m * 8);
    s.st.w = (unsigned long long*)take(s.tiles * 64ull);
    s.st.ticket = (uint32_t*)take(8);
    s.tmp_bytes = sort_tmp_bytes(n, cap_bits + 1u);
    s.tmp = take(s.tmp_bytes);
    return s;
}

unsigned long long* time_key_array(void* scratch) { return static_cast<unsigned long long*>(scratch); }
hipError_t launch_time_prepare(void* scratch, uint32_t n_slots, hipStream_t s) {
    return n_slots ? hipMemsetAsync(scratch, 0xFF, (size_t)n_slots * 8u, s) : hipSuccess;  // "no flow"
}

hipError_t launch_time_update(const FlowParams& p, uint32_t n_slots, uint64_t cap, FlowTime* plane,
                              const unsigned long long* ts, void* scratch, hipStream_t st) {
    if (n_slots == 0u) return hipSuccess;
    uint32_t bits = 0;
    while ((1ull << bits) < cap) ++bits;
    const uint32_t c = (uint32_t)cap;  // (<= 2^25: the sort key's "no flow" value is cap itself)
    TimeScratch s = carve(scratch, n_slots, bits);
    hipError_t e;
    size_t tb = s.tmp_bytes;
    e = time_sort(s.tmp, tb, s.kv, s.ks, s.tsort, ts, c, n_slots, bits + 1u, st);
    if (e != hipSuccess) return e;
    // the tiles' status words and the ticket after them (carve keeps them adjacent): one memset
    if ((e = hipMemsetAsync(s.st.w, 0, (size_t)((char*)s.st.ticket - (char*)s.st.w) + 8u, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_time_runs, dim3(s.tiles), dim3(kRunThreads), 0, st, s.ks, n_slots, c, p.table,
                       plane, ts, s.tsort, p.batch, s.st);
    return hipGetLastError();
}

hipError_t launch_time_remap(const FlowTime* old, const uint32_t* remap, unsigned long long old_cap, FlowTime* nw,
                             hipStream_t s) {
    const unsigned long long g = (old_cap + kTmThreads - 1) / kTmThreads;
    hipLaunchKernelGGL(k_time_remap, dim3((uint32_t)g), dim3(kTmThreads), 0, s, old, remap, old_cap, nw);
    return hipGetLastError();
}

hipError_t launch_time_export(const FlowSlot* table, const FlowTime* plane, unsigned long long cap, fb_flow_time* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > 1024ull) g = 1024ull;
    if (g == 0ull) g = 1ull;
    hipLaunchKernelGGL(k_time_export, dim3((uint32_t)g), dim3(256), 0, s, table, plane, cap, out, out_cap, d_n);
    return hipGetLastError();
}

}  // namespace fbk
