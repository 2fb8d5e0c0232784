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
// stable sort of the batch's records by table slot (they arrive in packet order) and two device-wide
// inclusive scans -- the latest reset / end / run head at or before each packet (max of index + 1:
// a flow's packets are contiguous, so a value below its run's head means "none in this batch, use
// the time plane") and the running end count -- give every packet its inputs, a second scan the
// accepted interarrival sum, and the run's last packet writes the flow's new FlowTime:
//   K_keys   one thread per record slot: the record's key (record or update entry), its table slot
//            (probe of the updated table), sort key = slot (cap: no flow -> sorts last), value =
//            pkt_index << 1 | P
//   sort     rocPRIM LSD radix sort of (slot, value) pairs over log2(cap) + 1 bits (stable: the
//            packet order inside a slot stays)
//   K_flags  per sorted packet: its capture time, T, in, end, reset (its own and its predecessor's:
//            the predecessor's `in` needs the packet before that), the scan input
//   scan 1   (head, reset, end) max, end count sum
//   K_ia     per packet that ends a segment after an earlier end: the interarrival term (ms) if
//            accepted (>= 0, src/packets.rs:165), and the divisor segment_count - 1 then
//   scan 2   accepted ms sum, last accepted index max
//   K_write  per run's last packet: the flow's FlowTime (start / end from the table's positions of
//            this call, last = the run's last packet)
// Bytes per record: 8 B (sort pairs, 3 passes of 2 x 8 B) + 8 B timestamp + 16 + 16 B scan words
// + the table probe (a 128-B slot line) -- an auxiliary pass, not the headline path.
#include <cstring>  // (rocPRIM's texture-cache iterator needs memset declared)

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "fb_internal.h"

namespace fbk {

namespace {

constexpr uint32_t kTmThreads = 256;
constexpr uint32_t kTmInvalidDiv = 0u;

// chrono's (a - b).num_milliseconds(): the signed difference truncated toward zero
__device__ __forceinline__ long long ms_between(unsigned long long a, unsigned long long b) {
    return ((long long)a - (long long)b) / 1000000ll;
}
__device__ __forceinline__ bool timeout_of(unsigned long long now, unsigned long long last) {
    return ms_between(now, last) >= (long long)FB_SEGMENT_TIMEOUT_MS;
}

struct ScanA {  // scan 1 word: index + 1 of the latest run head / reset / end at or before, ends so far
    uint32_t h, r, e, c;
};
struct ScanAOp {
    __device__ __host__ ScanA operator()(const ScanA& a, const ScanA& b) const {
        return ScanA{a.h > b.h ? a.h : b.h, a.r > b.r ? a.r : b.r, a.e > b.e ? a.e : b.e, a.c + b.c};
    }
};
struct ScanB {  // scan 2 word: accepted interarrival ms so far, index + 1 of the latest accepted term
    long long s;
    uint32_t a, pad;
};
struct ScanBOp {
    __device__ __host__ ScanB operator()(const ScanB& x, const ScanB& y) const {
        return ScanB{x.s + y.s, x.a > y.a ? x.a : y.a, 0u};
    }
};

// per sorted packet flags (K_flags)
constexpr uint8_t kFP = 1u, kFT = 2u, kFIn = 4u, kFHead = 8u, kFIns = 16u, kFEnd = 32u, kFInPrev = 64u;

// The table slot of `key` (the update just inserted every key it took), or `cap` if absent (a record
// the table could not take: its flow is not in the table).
__device__ __forceinline__ uint32_t table_slot(const FlowSlot* T, uint32_t part_shift, const uint32_t key[10],
                                               uint32_t cap) {
    const unsigned long long h = flow_hash_words(key);
    const uint32_t part = part_of(h, part_shift);
    const uint32_t want = (uint32_t)h | 2u;
    uint32_t j = (uint32_t)h & (kFlowSlots - 1u);
    const FlowSlot* P = T + (size_t)part * kFlowSlots;
    for (uint32_t probe = 0; probe < kFlowSlots; ++probe) {
        const FlowSlot& s = P[j];
        const uint32_t tag = s.tag;
        if (tag == 0u) return cap;
        if (tag == want) {
            bool eq = (s.key[9] & 0xFFFFu) == (key[9] & 0xFFFFu);
#pragma unroll
            for (int k = 0; k < 9; ++k) eq &= s.key[k] == key[k];
            if (eq) return part * kFlowSlots + j;
        }
        j = (j + 1u) & (kFlowSlots - 1u);
    }
    return cap;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kTmThreads) void k_time_keys(const FlowParams P, uint32_t n, uint32_t cap,
                                                          uint32_t* keys, uint32_t* vals) {
    const uint32_t i = blockIdx.x * kTmThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t nrec = batch_records(P);
    bool ok = i < nrec;
    uint32_t w = i;
    if (ok && P.rec_part) {  // update entries of the fused parse (fb_internal.h UpdEnt)
        ok = !P.seg || (i & 63u) < (P.seg[i >> 6] & 0xFFFFu);
        const uint32_t pw = ok ? P.rec_part[i] : 0u;
        w = (i >> 6) * kUpdUnitsPerSeg + ((pw >> kRecUnitShift) & 127u) | ((pw & kRecV6) ? kEntV6 : 0u);
    } else if (ok) {
        ok = slot_valid(P, i);
    }
    uint32_t key = cap, val = 0u;
    if (ok) {
        uint4 e[4];
        if (P.rec_part) {
            uint4 r[4];
            raw_entry(P, w, r);
            entry_of(true, r, w, e);
        } else {
            uint4 r[4];
            raw_entry(P, w, r);
            entry_of(false, r, w, e);
        }
        const uint32_t k[10] = {e[0].x, e[0].y, e[0].z, e[0].w, e[1].x, e[1].y, e[1].z, e[1].w, e[2].x, e[2].y & 0xFFFFu};
        const uint32_t pkt = e[3].x, hinfo = e[3].z;
        const uint32_t flags = (hinfo >> 8) & 0xFFu;
        const bool has_flags = (hinfo >> 16) & 1u;
        const bool psh = has_flags && (k[9] & 0xFFu) == 6u && (flags & kTcpPsh);
        key = table_slot(P.table, P.part_shift, k, cap);
        val = pkt << 1 | (psh ? 1u : 0u);
    }
    keys[i] = key;
    vals[i] = val;
}

// The sorted packets: capture time, T / in / end / reset flags and the scan-1 input.
__global__ __launch_bounds__(kTmThreads) void k_time_flags(const uint32_t* keys, const uint32_t* vals, uint32_t n,
                                                           uint32_t cap, const FlowSlot* T, const FlowTime* plane,
                                                           const unsigned long long* ts, uint32_t batch,
                                                           unsigned long long* t_out, uint8_t* f_out, ScanA* a_out) {
    const uint32_t i = blockIdx.x * kTmThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = keys[i];
    if (s >= cap) {  // no flow: neutral scan word
        f_out[i] = 0u;
        a_out[i] = ScanA{0u, 0u, 0u, 0u};
        return;
    }
    const unsigned long long pos_hi = (unsigned long long)batch << 32;
    // element j's (T, in, insert) given its predecessor; `hd` whether j heads its run
    auto state = [&](uint32_t j, bool hd, unsigned long long tj, unsigned long long tprev_elem, bool& T_, bool& in_,
                     bool& ins_) {
        const bool P_ = vals[j] & 1u;
        ins_ = false;
        unsigned long long tprev = tprev_elem;
        if (hd) {
            ins_ = T[s].first_seen == (pos_hi | (vals[j] >> 1));  // the flow's insert is this packet
            tprev = plane[s].last_activity_ns;
        }
        T_ = !ins_ && timeout_of(tj, tprev);
        in_ = ins_ ? !P_ : (T_ || !P_);
    };
    const bool head = i == 0u || keys[i - 1u] != s;
    const unsigned long long t = ts[vals[i] >> 1];
    const unsigned long long t1 = head ? 0ull : ts[vals[i - 1u] >> 1];
    bool Ti, ini, insi;
    state(i, head, t, t1, Ti, ini, insi);
    bool in_prev;
    if (head) {
        in_prev = insi ? false : plane[s].in_segment != 0u;
    } else {
        const bool head1 = i == 1u || keys[i - 2u] != s;
        const unsigned long long t2 = head1 ? 0ull : ts[vals[i - 2u] >> 1];
        bool T1, in1, ins1;
        state(i - 1u, head1, t1, t2, T1, in1, ins1);
        in_prev = in1;
    }
    const bool P_ = vals[i] & 1u;
    const bool end = insi ? P_ : (P_ || (in_prev && Ti));
    const bool reset = insi || Ti || !in_prev;
    t_out[i] = t;
    f_out[i] = (uint8_t)((P_ ? kFP : 0u) | (Ti ? kFT : 0u) | (ini ? kFIn : 0u) | (head ? kFHead : 0u) |
                         (insi ? kFIns : 0u) | (end ? kFEnd : 0u) | (in_prev ? kFInPrev : 0u));
    a_out[i] = ScanA{head ? i + 1u : 0u, reset ? i + 1u : 0u, end ? i + 1u : 0u, end ? 1u : 0u};
}

// Interarrival terms: at an end that follows an earlier end (in this batch or the plane's).
__global__ __launch_bounds__(kTmThreads) void k_time_ia(const uint32_t* keys, uint32_t n, uint32_t cap,
                                                        const FlowTime* plane, const unsigned long long* t,
                                                        const uint8_t* f, const ScanA* A, ScanB* b_out,
                                                        uint32_t* div) {
    const uint32_t i = blockIdx.x * kTmThreads + threadIdx.x;
    if (i >= n) return;
    ScanB out{0ll, 0u, 0u};
    const uint32_t s = keys[i];
    const uint8_t fl = f[i];
    if (s < cap && (fl & kFEnd) && !(fl & kFIns)) {
        const uint32_t H = A[i].h - 1u;  // the run's head
        const bool ins_run = f[H] & kFIns;
        const ScanA prev = i > H ? A[i - 1u] : ScanA{0u, 0u, 0u, 0u};
        // previous end: in this run before i, else the plane's (a new flow's run has none before)
        unsigned long long prev_end = FB_SEEN_NONE;
        if (prev.e > H) prev_end = t[prev.e - 1u];
        else if (!ins_run) prev_end = plane[s].last_segment_end_ns;
        if (prev_end != FB_SEEN_NONE) {
            unsigned long long start;  // current_segment_start as of packet i (src/packets.rs:151-154)
            if (!(fl & kFInPrev)) start = t[i];
            else if (prev.r > H) start = t[prev.r - 1u];
            else start = plane[s].current_segment_start_ns;
            const long long ia = ms_between(start, prev_end);
            if (ia >= 0) {  // (double)ia / 1000.0 >= 0.0 (src/packets.rs:165)
                const uint32_t before = (i > H ? prev.c - (H > 0u ? A[H - 1u].c : 0u) : 0u) +
                                        (ins_run ? 0u : plane[s].segment_count);
                out = ScanB{ia, i + 1u, 0u};
                div[i] = before;  // segment_count after this end, minus 1
            }
        }
    }
    b_out[i] = out;
}

// Each run's last packet: the flow's new time record.
__global__ __launch_bounds__(kTmThreads) void k_time_write(const uint32_t* keys, const uint32_t* vals, uint32_t n,
                                                           uint32_t cap, const FlowSlot* T, FlowTime* plane,
                                                           const unsigned long long* ts, uint32_t batch,
                                                           const unsigned long long* t, const uint8_t* f,
                                                           const ScanA* A, const ScanB* B, const uint32_t* div) {
    const uint32_t i = blockIdx.x * kTmThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = keys[i];
    if (s >= cap || (i + 1u < n && keys[i + 1u] == s)) return;  // not a run's last packet
    const uint32_t H = A[i].h - 1u;
    const bool ins = f[H] & kFIns;
    FlowTime o;
    if (ins) {
        o.start_time_ns = t[H];
        o.end_time_ns = FB_SEEN_NONE;
        o.current_segment_start_ns = t[H];
        o.last_segment_end_ns = FB_SEEN_NONE;
        o.total_segment_interarrival_ms = 0ll;
        o.segment_interarrival_div = kTmInvalidDiv;
        o.segment_count = 0u;
    } else {
        o = plane[s];
    }
    const ScanA a = A[i];
    const uint32_t c0 = H > 0u ? A[H - 1u].c : 0u;
    o.segment_count += a.c - c0;
    if (a.r > H) o.current_segment_start_ns = t[a.r - 1u];
    if (a.e > H) o.last_segment_end_ns = t[a.e - 1u];
    const long long s0 = H > 0u ? B[H - 1u].s : 0ll;
    o.total_segment_interarrival_ms += B[i].s - s0;
    if (B[i].a > H) o.segment_interarrival_div = div[B[i].a - 1u];
    o.last_activity_ns = t[i];
    o.in_segment = (f[i] & kFIn) ? 1u : 0u;
    // end_time at the flow's first FIN/RST, which the update placed in end_seen (src/packets.rs:195-198)
    const unsigned long long es = T[s].end_seen;
    if (es != FB_SEEN_NONE && (es >> 32) == (unsigned long long)batch && o.end_time_ns == FB_SEEN_NONE)
        o.end_time_ns = ts[es & 0xFFFFFFFFull];
    o.reserved[0] = o.reserved[1] = o.reserved[2] = 0u;
    o.slot = 0u;
    plane[s] = o;
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
struct TimeScratch {
    uint32_t *keys, *keys2, *vals, *vals2, *div;
    unsigned long long* t;
    uint8_t* f;
    ScanA* a;
    ScanA* a2;
    ScanB* b;
    ScanB* b2;
    void* tmp;
    size_t tmp_bytes;
};
static size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

static size_t lib_tmp_bytes(uint32_t n, uint32_t bits) {
    size_t a = 0, b = 0, c = 0;
    rocprim::radix_sort_pairs(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                              (uint32_t*)nullptr, n, 0u, bits, (hipStream_t)0);
    rocprim::inclusive_scan(nullptr, b, (ScanA*)nullptr, (ScanA*)nullptr, n, ScanAOp(), (hipStream_t)0);
    rocprim::inclusive_scan(nullptr, c, (ScanB*)nullptr, (ScanB*)nullptr, n, ScanBOp(), (hipStream_t)0);
    return std::max(a, std::max(b, c));
}

uint64_t time_scratch_bytes(uint32_t n, uint32_t cap_bits) {
    const size_t m = std::max<uint32_t>(n, 1u);
    return al256(m * 4) * 5 + al256(m * 8) + al256(m) + al256(m * sizeof(ScanA)) * 2 + al256(m * sizeof(ScanB)) * 2 +
           al256(lib_tmp_bytes(n, cap_bits + 1u));
}

static TimeScratch carve(void* base, uint32_t n, uint32_t cap_bits) {
    char* p = static_cast<char*>(base);
    const size_t m = std::max<uint32_t>(n, 1u);
    auto take = [&](size_t b) { char* q = p; p += al256(b); return q; };
    TimeScratch s;
    s.keys = (uint32_t*)take(m * 4);
    s.keys2 = (uint32_t*)take(m * 4);
    s.vals = (uint32_t*)take(m * 4);
    s.vals2 = (uint32_t*)take(m * 4);
    s.div = (uint32_t*)take(m * 4);
    s.t = (unsigned long long*)take(m * 8);
    s.f = (uint8_t*)take(m);
    s.a = (ScanA*)take(m * sizeof(ScanA));
    s.a2 = (ScanA*)take(m * sizeof(ScanA));
    s.b = (ScanB*)take(m * sizeof(ScanB));
    s.b2 = (ScanB*)take(m * sizeof(ScanB));
    s.tmp_bytes = lib_tmp_bytes(n, cap_bits + 1u);
    s.tmp = take(s.tmp_bytes);
    return s;
}

hipError_t launch_time_update(const FlowParams& p, uint32_t n_slots, uint64_t cap, FlowTime* plane,
                              const unsigned long long* ts, void* scratch, hipStream_t st) {
    if (n_slots == 0u) return hipSuccess;
    uint32_t bits = 0;
    while ((1ull << bits) < cap) ++bits;
    const uint32_t c = (uint32_t)cap;  // (<= 2^25: the sort key's "no flow" value is cap itself)
    TimeScratch s = carve(scratch, n_slots, bits);
    const uint32_t g = (n_slots + kTmThreads - 1u) / kTmThreads;
    hipLaunchKernelGGL(k_time_keys, dim3(g), dim3(kTmThreads), 0, st, p, n_slots, c, s.keys, s.vals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = s.tmp_bytes;
    e = rocprim::radix_sort_pairs(s.tmp, tb, s.keys, s.keys2, s.vals, s.vals2, n_slots, 0u, bits + 1u, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_time_flags, dim3(g), dim3(kTmThreads), 0, st, s.keys2, s.vals2, n_slots, c, p.table, plane, ts,
                       p.batch, s.t, s.f, s.a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = s.tmp_bytes;
    e = rocprim::inclusive_scan(s.tmp, tb, s.a, s.a2, n_slots, ScanAOp(), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_time_ia, dim3(g), dim3(kTmThreads), 0, st, s.keys2, n_slots, c, plane, s.t, s.f, s.a2, s.b,
                       s.div);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = s.tmp_bytes;
    e = rocprim::inclusive_scan(s.tmp, tb, s.b, s.b2, n_slots, ScanBOp(), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_time_write, dim3(g), dim3(kTmThreads), 0, st, s.keys2, s.vals2, n_slots, c, p.table, plane, ts,
                       p.batch, s.t, s.f, s.a2, s.b2, s.div);
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
