// fb_internal.h -- definitions shared by the gfx950 kernels and the C-ABI host code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flodbadd_gpu.h"

namespace fbk {

// Launch scratch (one allocation per context): tick[8 * FB_MAX_SEG_BATCHES] u64, k_parse_seg's
// packed per-batch stats words; the block that completes a word zeroes it for the next launch.
constexpr uint32_t kTickWords = 8u * FB_MAX_SEG_BATCHES;

// Device-resident configuration (uploaded lazily, stream-ordered, before a launch).
struct LanV6 {
    uint32_t net[4];
    uint32_t mask[4];
};
// The parse kernel copies the first kCfgLdsBytes (header + service bitmap) into LDS; the
// tables behind them are read from global memory by uniform loops (only when non-empty).
struct DevConfig {
    uint32_t filter;
    uint32_t n_lan_v6;
    uint32_t n_own;
    uint32_t pad;
    uint32_t service_bitmap[FB_SERVICE_BITMAP_BYTES / 4];  // bit p <=> name(p) != ""
    LanV6 lan_v6[FB_MAX_LAN_V6];
    fb_ip own[FB_MAX_OWN_IPS];
};
constexpr uint32_t kCfgLdsBytes = 16u + FB_SERVICE_BITMAP_BYTES;

// Per-launch parameters of k_parse_seg beside its batch descriptors (SegBatches).
struct ParseParams {
    const fb_parsed_pkt* parsed;  // parsed-packet instance (fb_process_parsed*): the input records
    uint32_t n;                   // parsed-packet instance: records in `parsed`
    uint32_t part_shift;          // FlowParams::part_shift of the context's table
    const DevConfig* cfg;
    unsigned long long* tick;     // [kTickWords] packed stats words, 8 per batch of the launch
    uint32_t* error;              // this launch's error word (launch parity); set by the flow kernels
    uint32_t* error_next;         // the other parity's word, zeroed by this launch for the next one
    uint32_t* rec_part;           // one batch: partition of each SESSION record slot, or nullptr
    uint4* rec_ent;               // with rec_part: the update entry of each SESSION record slot
                                  // (UpdEnt, 64-B units) -- what the table update reads
    uint32_t no_records;          // with rec_part: SESSION records not stored (the table is the
                                  // output; DNS records, counts, classes and stats still are)
    const unsigned long long* pre;  // dense pass 2: per segment n_session | n_dns << 32 before it
    fb_pkt_out* dense_out;        // dense pass 2: batch-wide SESSION records (or nullptr)
    fb_dns_out* dense_dns;        // dense pass 2: batch-wide DNS records (or nullptr)
    // k_parse_dense (single-pass dense output): per-tile look-back words, the launch's 8-bit
    // epoch, the number of tiles, and the polls a look-back waits for a predecessor's word before
    // computing that tile's sums itself
    unsigned long long* dstatus;
    uint32_t dep;
    uint32_t ntiles;
    uint32_t steal_polls;
    // fault injection for the tests (FB_DENSE_OFFSET_SKEW at fb_create, 0 otherwise): added to every
    // tile offset k_parse_dense hands its copies, as a corrupted look-back word would be
    unsigned long long dn_skew;
#if defined(FB_DN_TRACE) || defined(FB_SEG_TRACE)
    // diagnostic builds: k_parse_dense / k_parse_seg timings (fb_parse.hip, kDnTr* / kSegTr*)
    unsigned long long* dtrace;
#endif
};
// 16 / 8 bytes at a 4-B aligned address: 56-B records (fb_pkt_out, fb_parsed_pkt) are only 8-B
// aligned at odd indices, so a uint4 dereference there would claim an alignment the data lacks
// (undefined behaviour the compiler did act on: a k_parse_seg instance read a parsed record's
// words rotated by one until its loads went through byte offsets).
__device__ __forceinline__ uint4 ld_u4(const uint32_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ uint2 ld_u2(const uint32_t* p) {
    uint2 v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// is_lan_ip, src/ip.rs:55-156, 199-242.
__device__ __forceinline__ bool lan_v4(uint32_t v) {
    uint32_t a = v >> 24, b = (v >> 16) & 0xffu;
    return v == 0u || v == 0xffffffffu || a == 127u || (v >> 28) == 0xEu || (v >> 16) == 0xA9FEu ||
           a == 10u || (a == 172u && b >= 16u && b <= 31u) || (v >> 16) == 0xC0A8u;
}
__device__ __forceinline__ bool lan_v6(const DevConfig* c, const DevConfig* g, const uint32_t w[4]) {
    uint32_t s0 = w[0] >> 16;
    if ((w[0] | w[1] | w[2] | w[3]) == 0u) return true;                       // ::
    if ((w[0] | w[1] | w[2]) == 0u && w[3] == 1u) return true;                // ::1
    if ((s0 & 0xffc0u) == 0xfe80u || (s0 & 0xff00u) == 0xff00u || (s0 & 0xfe00u) == 0xfc00u)
        return true;                                                          // fe80::/10 ff00::/8 fc00::/7
    const uint32_t nl = c->n_lan_v6;                                          // uniform loop
    for (uint32_t i = 0; i < nl; ++i) {
        const LanV6& e = g->lan_v6[i];
        if ((w[0] & e.mask[0]) == e.net[0] && (w[1] & e.mask[1]) == e.net[1] &&
            (w[2] & e.mask[2]) == e.net[2] && (w[3] & e.mask[3]) == e.net[3])
            return true;
    }
    return false;
}
__device__ __forceinline__ bool own_ip(const DevConfig* c, const DevConfig* g, uint32_t fam, const uint32_t w[4]) {
    const uint32_t no = c->n_own;
    bool hit = false;
    for (uint32_t i = 0; i < no; ++i) {
        const fb_ip& o = g->own[i];
        hit |= o.family == fam && o.addr[0] == w[0] && o.addr[1] == w[1] && o.addr[2] == w[2] &&
               o.addr[3] == w[3];
    }
    return hit;
}

// Batches of one k_parse_seg launch (fb_parse_classify_seg_batches_dev): the launch streams over
// the concatenation of their segments; batch k owns global segments [seg_start, next seg_start).
constexpr uint32_t kMaxSegBatches = FB_MAX_SEG_BATCHES;
struct SegBatch {
    const uint8_t* frames;
    const uint32_t* offsets;
    fb_pkt_out* out;
    uint32_t* seg;
    uint8_t* cls;
    fb_batch_stats* stats;
    uint32_t n;
    uint32_t frames_bytes;
    uint32_t seg_start;
    uint32_t pad;
};
struct SegBatches {
    SegBatch b[kMaxSegBatches];
    uint32_t count;
    uint32_t total_segs;
};

// Flow (session) table, partitioned for owner-computes updates (fb_flow.hip):
//   capacity = P partitions x kFlowSlots slots; a key's partition is the top log2(P) bits of its
//   64-bit hash, its home slot inside the partition the low bits (linear probing wraps inside
//   the partition).  One workgroup owns one partition per batch and updates it in LDS, so the
//   upsert needs no global atomics.
//   Slot (128 B): tag (0 empty, 1 being inserted [LDS only], else the hash's low word | 2) and
//   segment_count in one u64 (so K2 adds PSH packets to the high half with one LDS atomic), 40-B
//   key, 6 counters in fb_flow_rec order, then the ordered state: first / last / end positions
//   ((update call << 32) | pkt_index, FB_SEEN_NONE), hist_len, hist_mask | in_segment << 14 |
//   dst_service << 15 | conn_state << 16 | session flags << 20 | end_mask << 24.
#ifndef FB_FLOW_SLOTS
#define FB_FLOW_SLOTS 512
#endif
constexpr uint32_t kFlowSlots = FB_FLOW_SLOTS;   // slots per partition: 64 KiB LDS slice
constexpr uint32_t kFlowMaxParts = 65536;        // K1 histogram in LDS (u16 counters past 16,384
                                                 // partitions): capacity <= 2^25 slots (4 GiB)
constexpr uint32_t kFlowPackedParts = 16384;     // more partitions than this: K1 counts in u16 halves
#ifndef FB_FLOW_CHUNK
#define FB_FLOW_CHUNK 20480  // 512 chunks per 10M-record C4 batch = one wave of the 512 K1 workgroups
                             // resident at once (16,384: 640 chunks, a 128-workgroup second wave;
                             // C4 update 0.664 -> 0.623 ms, tools/chunk_ab.sh)
#endif
#ifndef FB_K1_THREADS
#define FB_K1_THREADS 1024
#endif
constexpr uint32_t kFlowChunk = FB_FLOW_CHUNK;   // records per bucketing workgroup (K1)
constexpr uint32_t kFlowK1Threads = FB_K1_THREADS;
#ifndef FB_K2_THREADS
#define FB_K2_THREADS 512  // two 8-wave workgroups per CU (68 KiB LDS each): 1.26 ms for the C4 update vs 1.38 at one 16-wave workgroup
#endif
constexpr uint32_t kFlowK2Threads = FB_K2_THREADS;
constexpr uint64_t kFlowMaxCapacity = (uint64_t)kFlowSlots * kFlowMaxParts;
struct FlowSlot {
    uint32_t tag;               // 0 empty, else (uint32_t)fb_flow_hash | 2
    uint32_t segment_count;     // SessionStats.segment_count (TCP packets with PSH, src/packets.rs:140-160, 414-420)
    uint32_t key[10];
    unsigned long long cnt[6];  // outbound_bytes, inbound_bytes, orig_pkts, resp_pkts,
                                // orig_ip_bytes, resp_ip_bytes
    unsigned long long first_seen, last_seen, end_seen;
    uint32_t hist_len;
    uint32_t hist_state;        // hist_mask (FB_HIST_CHARS bits) | in_segment << 14 | dst_service << 15 |
                                // conn_state << 16 (4 bits) | session flags << 20 (fb_session_flags 0-3,
                                // set at insert) | end_mask << 24
};
constexpr uint32_t kStateInSegment = 1u << 14;  // hist_state: SessionStats.in_segment
constexpr uint32_t kTcpPsh = 0x08u;             // TCP_PSH, src/packets.rs:26
static_assert(sizeof(FlowSlot) == 128, "flow slot is 128 B");
// Capture-time state per table slot on a timed context (the "time plane", fb_time.hip).
using FlowTime = fb_flow_time;
static_assert(sizeof(FlowTime) == 64, "one 64-B time record per slot");
// Bucketed update entry (K1 -> K2): canonical key with the originator flag in bit 16 of
// word 9 (the key's padding), L4 payload bytes, IP bytes, then the record's pkt_index, its
// record slot (the batch order K2 orders the history by), hist_char | tcp_flags << 8 |
// has_flags << 16, and the low word of the key's hash.
struct FlowEntry {
    uint32_t key[10];
    uint32_t packet_length;
    uint32_t ip_packet_length;
    uint32_t pkt_index;
    uint32_t rec;
    uint32_t hist;
    uint32_t hash_lo;  // low word of fb_flow_hash(key)
};
static_assert(sizeof(FlowEntry) == 64, "flow entry is 64 B");
// A combined entry (k_flow_combine: the records of one key in one hot bucketing group) takes two
// consecutive FlowEntry units.  Head: key[0..8], key[9] | kEntCombined, first rec, last rec,
// combined id, end rec (first FIN/RST, ~0 none), hist count | hist mask << 16, hash_lo.  Tail:
// outbound, inbound, orig ip, resp ip bytes (u64), orig | resp pkts << 16, kEntTail, first rec
// of S s H h (~0 none), records, session flags | end char bit << 8 | last record's PSH << 15 |
// PSH records << 16.
constexpr uint32_t kEntCombined = 1u << 17;  // in key[9] (bit 16 is the originator)
constexpr uint32_t kEntTail = 1u << 18;
constexpr uint32_t kRecFlowCombined = 0x80000000u;  // e_sort position word: combined id, slot in agg_slot
// entries[] word: the record slot (< 2^27) | its history code << 27 (0: no history character --
// not TCP --, else 1 + the character's FB_HIST_CHARS index), or kIdxCombined | a combined id
constexpr uint32_t kIdxCombined = 0x80000000u;
constexpr uint32_t kEntRecMask = 0x07FFFFFFu;
constexpr uint32_t kEntCodeShift = 27;
// K2's history word of a plain entry: its table slot within the partition (9 bits), history code
// (4 bits, 0: none) << 9, record slot within its bucketing chunk (15 bits) << 13; 0 for an entry
// the table could not take.
static_assert(FB_FLOW_SLOTS == 512 && FB_FLOW_CHUNK <= 32768, "hist_word field widths");
__device__ __forceinline__ uint32_t hist_word(uint32_t slot_local, uint32_t code, uint32_t rec) {
    return slot_local | (code & 15u) << 9 | (rec % kFlowChunk) << 13;
}
__device__ __forceinline__ uint32_t hist_word(uint32_t slot_local, uint32_t entry_word) {
    return hist_word(slot_local, entry_word >> kEntCodeShift, entry_word & kEntRecMask);
}

// fb_flow_hash of a 40-B session_key (10 words, word 9 = protocol | family << 8) and the
// partition it falls in (top bits).
__host__ __device__ inline unsigned long long flow_hash_words(const uint32_t k[10]) {
    unsigned long long h = 0x9E3779B97F4A7C15ull;
    for (int j = 0; j < 10; j += 2) {
        const unsigned long long w = (unsigned long long)k[j] | ((unsigned long long)k[j + 1] << 32);
        h ^= w;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    return h;
}

__device__ __forceinline__ uint32_t part_of(unsigned long long h, uint32_t shift) {
    return shift >= 64u ? 0u : (uint32_t)(h >> shift);
}

struct FlowParams {
    const fb_pkt_out* recs;
    const uint32_t* seg;        // non-null: recs are 64-record segments, record slot i valid iff
                                // (i & 63) < (seg[i >> 6] & 0xFFFF); n_slots slots in all
    uint32_t n_slots;
    fb_batch_stats* stats;      // n_session read from here; new/updated accumulated
    FlowSlot* table;
    uint32_t* entries;          // [max_recs] bucketed by partition: the record slot of each entry,
                                // or kIdxCombined | id of a k_flow_combine entry in `comb`
    FlowEntry* comb;            // [2 * comb_cap] combined entries (head + tail unit each)
    uint32_t comb_cap;
    uint32_t* rows;             // [chunks][parts]  start | count << 16, per bucketing chunk
    uint32_t* cols;             // [parts][chunk_stride] the same, transposed
    unsigned long long* partials;  // 4 per partition: new, updated, occupied slots after the update,
                                   // history characters | the partition's first hword index << 32
    uint32_t* error;
    uint32_t max_recs;          // scratch capacity in records
    uint32_t parts;             // P (power of two)
    uint32_t part_shift;        // 64 - log2(P) (64 when P == 1)
    uint32_t chunk_stride;      // >= ceil(max_recs / kFlowChunk)
    uint32_t batch;             // update call number since create / clear (positions' high word)
    uint32_t* rows_h;           // [chunks][parts] a combined group's row before k_flow_combine (K1c;
                                // the history reads its records from e_sort); a combined group's
                                // row in rows / cols has bit 15 set
    uint32_t* e_orig;           // [max_recs] K1c scratch: a combined group's original entry words
    uint2* e_sort;              // [max_recs] a combined group's records in record order (K1c): the
                                // original entry word, and the entry's new position or
                                // kRecFlowCombined | combined id
    uint32_t* hword;            // [max_recs] K2: a hist_word per entry it applied, each partition's in
                                // its entry order from partials[4 p + 3] >> 32 (coalesced writes)
    uint32_t* hcount;           // [capacity] history characters each slot got this update (K2)
    uint32_t* hot;              // [hot_cap] (chunk << 16 | part) groups K1 hands to k_flow_combine
    uint32_t* ctl;              // [4] hot groups, combined entries, hword entries, K1c's next group
                                // (reset by K1t)
    uint32_t* agg_slot;         // [max_recs / 2 + 1] table slot of each combined entry
    uint32_t hot_cap;
    uint32_t* part_base;        // [parts + 1] the history's output offset per partition (history)
    const uint32_t* rec_part;   // non-null: partition of each SESSION record slot, written by the
                                // segmented parse of the same batch (fb_process_seg_dev); K1's
                                // histogram pass then reads 4 B per record instead of the record
    const uint4* ent;           // non-null (with rec_part): the slots' update entries (UpdEnt), which
                                // K1c / K2 read instead of the records
    uint4* char_call = nullptr; // [capacity] per slot: the update call of the flow's first S, s, H, h
                                // (FB_CALL_NONE: none), for the multi-GPU merge (fb_flow_merge_dev)
    unsigned long long* tkv = nullptr;  // timed contexts: [record slots] K2 writes at each applied
                                // record's slot its table slot << 32 | pkt_index << 1 | PSH (~0u slot: not
                                // taken) -- the capture-time pass's sort input, in record (= packet) order
                                // (K2's own entry order is not: K1's scatter is not stable inside a
                                // chunk); K1c's combining is off then (every record a plain entry)
    uint32_t* order = nullptr;  // [parts + kK2Lead + 1] K2's partition order: per partition its entries
                                // (K1t's sums; bit 31: one of K2's leading workgroups takes it), the
                                // leading partitions, their count (zeroed by K1)
};
// K2's leading workgroups: the partitions with more than twice the mean entries (skewed popularity
// leaves flows K1c does not combine, up to ~18K entries in one partition under Zipf(1.1)), started
// before the rest instead of in partition order
constexpr uint32_t kK2Lead = 256;

// determine_conn_state, src/packets.rs:539-559, over FB_HIST_CHARS bits.
__host__ __device__ inline uint32_t conn_state_of(uint32_t m) {
    const bool S = m & 1u, H = m & 4u, h = m & 8u, F = m & 16u, f = m & 32u, R = m & 64u, r = m & 128u;
    if (S && H && F && f) return FB_CONN_SF;
    if (S && !h && !r) return FB_CONN_S0;
    if (R || r) return FB_CONN_REJ;
    if (S && H && !F && !f) return FB_CONN_S1;
    return FB_CONN_OTHER;
}

// A table slot as its export record (fb_flow_export, fb_flow_export_merge_dev).
__device__ __forceinline__ fb_flow_rec flow_rec_of(const FlowSlot& t, uint32_t slot) {
    fb_flow_rec r;
    __builtin_memcpy(&r.key, t.key, 40);
    r.outbound_bytes = t.cnt[0];
    r.inbound_bytes = t.cnt[1];
    r.orig_pkts = t.cnt[2];
    r.resp_pkts = t.cnt[3];
    r.orig_ip_bytes = t.cnt[4];
    r.resp_ip_bytes = t.cnt[5];
    r.first_seen = t.first_seen;
    r.last_seen = t.last_seen;
    r.end_seen = t.end_seen;
    r.hist_len = t.hist_len;
    r.hist_mask = (uint16_t)(t.hist_state & 0x1FFFu);
    r.conn_state = (uint8_t)((t.hist_state >> 16) & 0xFu);
    r.end_mask = (uint8_t)(t.hist_state >> 24);
    r.slot = slot;
    r.session_flags = ((t.hist_state >> 20) & 0xFu) | ((t.hist_state >> 15) & 1u) << 4;
    r.segment_count = t.segment_count;
    r.in_segment = (t.hist_state & kStateInSegment) ? 1u : 0u;
    r.reserved[0] = r.reserved[1] = r.reserved[2] = 0u;
    return r;
}

// Owner rank of a key in the multi-GPU merge (fb_flow_export_merge_dev): the high word of its
// fb_flow_hash scaled to [0, world).
__host__ __device__ inline uint32_t flow_owner(unsigned long long h, uint32_t world) {
    return (uint32_t)(((h >> 32) * (unsigned long long)world) >> 32);
}
// The fused parse's per-record word: the table partition (< kFlowMaxParts) in the low 16 bits,
// the record's history character in bits 16-23 and FB_META_HAS_FLAGS in bit 24 -- so the history
// keys kernel reads 4 B per record slot instead of the record.
constexpr uint32_t kRecPartMask = 0xFFFFu;
static_assert(kFlowMaxParts <= kRecPartMask + 1u, "partition ids fit the low half");

// Update entries (UpdEnt): what the fused parse (fb_process_seg[_async]_dev) hands the table update
// per SESSION record, packed in 32-B units -- one for an IPv4 key, two for an IPv6 key -- back to
// back in packet order inside a 4-KB region per 64-frame segment (128 units), so every line the
// parse writes is whole (per-slot 64-B units with the IPv4 half unwritten cost the C4 parse 1.5x:
// partial-line writes) and the update's random gathers read one aligned 32-B unit for an IPv4 key
// instead of a 56-B record that straddles a 128-B line 43 % of the time:
//   unit 0: key[0], key[4], key[8], key[9] | originator << 16     (addresses' first words, ports,
//                                                                   protocol | family << 8)
//           packet_length, ip_packet_length, pkt_index,
//           hinfo | rank << 26   (hinfo: hist_char | tcp_flags << 8 | has_flags << 16 | session
//                                 flags << 20 | dst_service << 24; rank: the record's slot in its
//                                 segment)
//   unit 1: key[1], key[2], key[3], key[5], key[6], key[7], 0, 0  (IPv6 only)
// The fused parse's per-slot word (rec_part) then holds partition | unit offset << 16 | IPv6 << 23,
// and the bucketing pass's index word is unit index | IPv6 << 28.  With entries the update orders a
// flow's packets by pkt_index (the frame index: monotone in packet order, within the record slots'
// bucketing chunk) instead of the record slot.
constexpr uint32_t kUpdUnitsPerSeg = 128;
constexpr uint32_t kUpdEntU4 = 4;                   // uint4 per record slot of the entry buffer (its size)
constexpr uint32_t kEntUnitMask = 0x0FFFFFFFu;      // index word: unit index
constexpr uint32_t kEntV6 = 1u << 28;               // index word: an IPv6 key (two units)
constexpr uint32_t kRecUnitShift = 16, kRecV6 = 1u << 23;  // rec_part fields
__host__ __device__ inline bool upd_ent_v6(uint32_t a_w) { return ((a_w >> 8) & 0xFFu) == 10u; }

// (shared by the table update, fb_flow.hip, and its capture-time pass, fb_time.hip)
// Record slots of the batch: dense -> n_session of the parse launch (read on the device);
// segmented -> every slot of every segment (invalid slots are skipped by slot_valid).
__device__ __forceinline__ uint32_t batch_records(const FlowParams& P) {
    // dense records whose offset scan expired (error bit 2, set only by k_seg_scan, which completes
    // before K1 starts: every workgroup of K1 / K1c / K2 reads the same value) never reach the table
    if (!P.seg && (__hip_atomic_load(P.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u)) return 0u;
    const unsigned long long n = P.seg ? (unsigned long long)P.n_slots : P.stats->n_session;
    return (uint32_t)min(n, (unsigned long long)P.max_recs);
}
__device__ __forceinline__ bool slot_valid(const FlowParams& P, uint32_t i) {
    return !P.seg || (i & 63u) < (P.seg[i >> 6] & 0xFFFFu);
}

// An entry word's record as the four uint4 of a plain FlowEntry (fb_internal.h): key words, key word
// 9 | originator << 16, packet_length, ip_packet_length, then pkt_index, rec, hist_char | tcp_flags
// << 8 | has_flags << 16 | session flags << 20, the low word of the key's hash.  `rec` orders a
// flow's packets: the record slot (entry word & kEntRecMask), or -- update entries from the fused
// parse (P.ent; the word is unit index | IPv6 << 28) -- the pkt_index.  Records are 56 B, so only
// 8-B aligned at odd slots: loaded through ld_u4 / ld_u2; an entry is one aligned 32-B unit (two
// for an IPv6 key).  The raw words are loaded first (raw_entry) and decoded when applied
// (entry_of), so K2 can keep loads in flight.
__device__ __forceinline__ void raw_entry(const FlowParams& P, uint32_t w, uint4 (&r)[4]) {
    if (P.ent) {
        const uint4* u = P.ent + (size_t)(w & kEntUnitMask) * 2u;
        r[0] = u[0];
        r[1] = u[1];
        if (w & kEntV6) {
            r[2] = u[2];
            r[3] = u[3];
        } else {
            r[2] = r[3] = make_uint4(0u, 0u, 0u, 0u);
        }
    } else {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(P.recs + (w & kEntRecMask));
        r[0] = ld_u4(q);
        r[1] = ld_u4(q + 4);
        r[2] = ld_u4(q + 8);
        const uint2 m = ld_u2(q + 12);  // flags | meta << 8 | hist_char << 16, pkt_index
        r[3] = make_uint4(m.x, m.y, 0u, 0u);
    }
}
__device__ __forceinline__ void entry_of(bool ent, const uint4 (&r)[4], uint32_t w, uint4 (&e)[4]) {
    if (ent) {  // UpdEnt units: A = r[0], B = r[1]; IPv6: r[2], r[3] (zero words for IPv4)
        const uint4 A = r[0], Bw = r[1], C = r[2], D = r[3];
        const uint32_t key[10] = {A.x, C.x, C.y, C.z, A.y, C.w, D.x, D.y, A.z, A.w & 0xFFFFu};
        e[0] = make_uint4(key[0], key[1], key[2], key[3]);
        e[1] = make_uint4(key[4], key[5], key[6], key[7]);
        e[2] = make_uint4(A.z, A.w & 0x1FFFFu, Bw.x, Bw.y);
        e[3] = make_uint4(Bw.z, Bw.z, Bw.w & 0x03FFFFFFu, (uint32_t)flow_hash_words(key));
    } else {
        const uint4 a = r[0], b = r[1], c = r[2];
        const uint32_t mx = r[3].x, my = r[3].y;
        const uint32_t key[10] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y & 0xFFFFu};
        const uint32_t meta = (mx >> 8) & 0xFFu;
        const uint32_t orig = (meta & FB_META_ORIGINATOR) ? 1u : 0u;
        const uint32_t hinfo = ((mx >> 16) & 0xFFu) | ((mx & 0xFFu) << 8) | ((meta & FB_META_HAS_FLAGS) ? 1u << 16 : 0u) |
                               ((meta >> 3) & 0x1Fu) << 20;  // FB_META_LOCAL_SRC .. DST_SERVICE -> fb_session_flags
        e[0] = a;
        e[1] = b;
        e[2] = make_uint4(c.x, (c.y & 0xFFFFu) | (orig << 16), c.z, c.w);
        e[3] = make_uint4(my, w & kEntRecMask, hinfo, (uint32_t)flow_hash_words(key));
    }
}
__device__ __forceinline__ void rec_entry(const FlowParams& P, uint32_t w, uint4 (&e)[4]) {
    uint4 r[4];
    raw_entry(P, w, r);
    entry_of(P.ent != nullptr, r, w, e);
}
// Resident queue-fed parse (fb_seg_queue_*, k_parse_seg_queue): the host control block lives in
// pinned, coherent host memory (the kernel reads it with system-scope loads); per ring slot the
// device keeps the batch's stats words (tick, 8 per slot) and the count of blocks done with it.
constexpr uint32_t kQueueMax = FB_QUEUE_MAX_DEPTH;
struct QueueHost {
    unsigned long long tail;    // batches submitted (host store, after the slot's descriptor)
    unsigned long long stop;    // host: no batch follows the submitted ones; the kernel exits when idle
    unsigned long long status;  // device: kQueueExpired -- a block waited idle_ticks for a batch and left
    unsigned long long pad[5];  // 0-2: an expired block's diagnostics; 3: the kernel's blocks, once all run
    unsigned long long cdone[kQueueMax];  // slot k % depth: k + 1 once batch k is complete (system store)
    fb_seg_batch desc[kQueueMax];         // slot k % depth: batch k (host stores)
};
constexpr unsigned long long kQueueExpired = 1ull;
constexpr uint32_t kQueueHeadWords = 128u;  // per slot: up to 8 counters, one 64-B line each
// The device side of the ring: ONE block at a time reads the host's tail over PCIe (poller: 0 free,
// else the polling block + 1) and copies the new descriptors here; every block reads these.
struct QueueDev {
    unsigned long long tail;   // batches whose descriptors are in desc[]
    unsigned long long stop;   // the host's stop word, as the last poll saw it with nothing left
    uint32_t poller;
    uint32_t pad[3];           // pad[0]: blocks started (the last one sets the host's pad[3])
    fb_seg_batch desc[kQueueMax];
};
struct QueueParams {
    const DevConfig* cfg;
    QueueHost* h;                  // device alias of the host control block
    QueueDev* d;                   // the device side (zeroed at create)
    unsigned long long* tick;      // [kQueueMax * 8] packed stats words per slot (k_parse_seg's format)
    uint32_t* blk_done;            // [kQueueMax] blocks that have finished the slot's batch
    uint32_t* head;                // [kQueueMax * kQueueHeadWords] the slot's chunk counters (k_parse_seg_queue)
    uint32_t* error;               // the queue's error word (copied into every batch's stats)
    uint32_t depth;                // ring slots: a power of two <= kQueueMax
    unsigned long long idle_ticks; // s_memrealtime ticks (100 MHz) a block waits for a batch before it leaves
    unsigned long long* trace;     // diagnostic builds (-DFB_QUEUE_TRACE): kQTraceWords x kQTraceN timings
};
// -DFB_QUEUE_TRACE (tools/build_variants.sh, never the product): per batch (k % kQTraceN) the
// real-time ticks of its publication in the device ring, the first block's descriptor load, the first
// and the last block's completion, and counts of the waves that drained and blocked before it and of
// the poller's host reads while it was awaited.
constexpr uint32_t kQTraceN = 1024u, kQTraceWords = 6u;
// then per block (up to kQTraceN blocks, 4 words): its completion ticks of batches kQtB0 and kQtB1,
// its HW_ID and XCC_ID registers
constexpr uint32_t kQtB0 = 100u, kQtB1 = 164u, kQTraceAll = kQTraceWords * kQTraceN + 4u * kQTraceN;
enum QTrace : uint32_t { kQtPub = 0, kQtFirst, kQtArr0, kQtDone, kQtDrain, kQtPolls };
// Workgroups per CU of the queue kernel (fb_seg_queue_create's note), and its waves per SIMD as the
// register budget is set: five at two workgroups (<= 102 VGPRs: no spills in the streaming loop, and a
// fifth wave's registers stay free on every SIMD for the blit and other kernels issued meanwhile)
#ifndef FB_QUEUE_BPC
#define FB_QUEUE_BPC 2
#endif
constexpr int kQueueWavesPerSimd = FB_QUEUE_BPC * 8 / 4 + 1;
// FB_QUEUE_SHARED: blocks = CUs / FB_QUEUE_SHARED_DIV (one per CU on that share of the CUs)
#ifndef FB_QUEUE_SHARED_DIV
#define FB_QUEUE_SHARED_DIV 8
#endif
hipError_t launch_parse_seg_queue(const QueueParams& q, uint32_t grid, hipStream_t s);
hipError_t occupancy_parse_seg_queue(int* blocks_per_cu);

// Launchers (fb_parse.hip / fb_compact.hip / fb_flow.hip).
// Which k_parse_seg instance: the segmented output; dense pass 1 (segment counts, classes, stats);
// dense pass 2 (records to batch-wide positions from the scanned counts, ParseParams::pre).
enum class SegPass { kSegments, kCount, kDenseOut };
hipError_t launch_parse_seg(const ParseParams& p, const SegBatches& sb, uint32_t grid, hipStream_t s,
                            SegPass pass = SegPass::kSegments);
hipError_t occupancy_parse_seg(int* blocks_per_cu);
uint32_t parse_seg_block_threads();
// Single-pass dense output of one frame batch (k_parse_dense): records, DNS records, classes and
// stats, tiles of parse_dense_tile_segs() segments (P.dstatus / dep / ntiles / steal_polls set by
// the caller).
hipError_t launch_parse_dense(const ParseParams& p, const SegBatch& b, uint32_t grid, hipStream_t s);
hipError_t occupancy_parse_dense(int* blocks_per_cu);
uint32_t parse_dense_tile_segs();
// Exclusive scan of segment count words into pre[nseg] (u64 n_session | n_dns << 32), and the
// dense copy of a segmented batch (fb_seg_compact_dev); out / dns may each be NULL.
// The scan's look-back scratch: seg_scan_tiles(nseg) epoch-tagged status words (zeroed whenever
// the 8-bit epoch wraps) and a ticket counter (zero between calls).
struct SegScanScratch {
    unsigned long long* status;
    uint32_t* ticket;
    uint32_t epoch;  // 1..255, a new one per call
    uint32_t* err;   // error word: bit 2 if a look-back spin ever expired
};
uint32_t seg_scan_tiles(uint32_t nseg);
hipError_t launch_seg_scan(const uint32_t* seg, uint32_t nseg, unsigned long long* pre, const SegScanScratch& sc,
                           hipStream_t s);
hipError_t launch_seg_compact(const fb_pkt_out* seg_out, const uint32_t* seg, uint32_t nseg, unsigned long long* pre,
                              const SegScanScratch& sc, fb_pkt_out* out, fb_dns_out* dns, hipStream_t s);
// One table update = launch_flow_bucket (K1 bucketing, K1c hot-group combine), launch_flow_transpose
// (K1t) and launch_flow_apply (K2; with transpose = true K1t first) -- separate calls so the
// pipelined path can put them on different streams.
hipError_t launch_flow_bucket(const FlowParams& p, uint32_t chunks, hipStream_t s, bool combine = true);
hipError_t launch_flow_transpose(const FlowParams& p, uint32_t chunks, hipStream_t s);
hipError_t launch_flow_combine(const FlowParams& p, hipStream_t s);
hipError_t launch_flow_apply(const FlowParams& p, uint32_t chunks, hipStream_t s, bool transpose = true);
// Table occupancy after an update, written by k_flow_finish into host-mapped memory so the host can
// decide to grow the table without waiting for the device: seq = the update's number (+1).
struct FlowMailbox {
    unsigned long long flows;     // occupied slots
    unsigned long long max_part;  // fullest partition (slots of kFlowSlots)
    unsigned long long new_flows; // keys the update inserted
    unsigned long long seq;       // written last
};
hipError_t launch_flow_finish(fb_batch_stats* stats, const unsigned long long* partials,
                              uint32_t nblk, uint32_t* error, FlowMailbox* mbox, unsigned long long seq,
                              hipStream_t s);
// Table growth by 2^k (1 <= k <= 5): every slot of `old` (old_parts partitions) re-inserted into `nw`
// (old_parts << k partitions, zeroed): a key's new partition is k more top bits of its hash, its home
// slot the same low bits; remap[old slot] = new slot (~0u for empty slots).
hipError_t launch_flow_grow(const FlowSlot* old, uint32_t old_parts, uint32_t k, uint32_t new_shift, FlowSlot* nw,
                            uint32_t* remap, const uint4* old_cc, uint4* new_cc, hipStream_t s);
// filter: fb_filter evaluated per flow at export time against `cfg` (is_local_session!,
// src/sessions.rs:660-672); FB_FILTER_ALL (cfg may be null) exports every flow.
// plane (timed contexts): segment_count / in_segment come from the flows' time records.
hipError_t launch_flow_export(const FlowSlot* table, unsigned long long cap, fb_flow_rec* out,
                              unsigned long long out_cap, unsigned long long* d_n,
                              hipStream_t s, uint32_t filter = FB_FILTER_ALL, const DevConfig* cfg = nullptr,
                              const FlowTime* plane = nullptr);
hipError_t launch_flow_count(const FlowSlot* table, unsigned long long cap,
                             unsigned long long* d_n, hipStream_t s);

// Multi-GPU merge (fb_merge.hip).  Export: every flow as an fb_flow_mrec grouped by owner rank
// (flow_owner), slot order inside each group, positions made global (+ shard_first), rec.slot = rank;
// d_counts[world] (u64) receives the group sizes.  scratch: merge_export_scratch_bytes(cap, world).
uint64_t merge_export_scratch_bytes(unsigned long long cap, uint32_t world);
// cmap (device, optional): per update call of this rank, global batch << 32 | the global index of its
// shard's first packet (fb_flow_export_merge_map_dev); null: call k = global batch k at shard_first.
hipError_t launch_merge_export(const FlowSlot* table, const uint4* char_call, unsigned long long cap, uint32_t world,
                               uint32_t rank, unsigned long long shard_first, const unsigned long long* cmap,
                               fb_flow_mrec* out, unsigned long long out_cap, unsigned long long* d_counts,
                               void* scratch, hipStream_t s);
// Routing: a rank's dense SESSION records (n_session of *stats, at most max_n) grouped by owner rank,
// stable, pkt_index += shard_first; ts_out[j] = ts[the record's frame] when ts is given.
uint64_t route_scratch_bytes(uint32_t max_n, uint32_t world);
hipError_t launch_route(const fb_pkt_out* recs, const fb_batch_stats* stats, uint32_t max_n, uint32_t world,
                        unsigned long long shard_first, const unsigned long long* ts, fb_pkt_out* out,
                        unsigned long long* ts_out, unsigned long long* d_counts, void* scratch, hipStream_t s);
// Merge: n records of one owner (every rank's group, rank order) -> one record per key in d_out (in
// the order of each key's first record), *d_n (u64) = keys.  scratch: merge_scratch_bytes(n).
uint64_t merge_scratch_bytes(unsigned long long n);
hipError_t launch_merge(const fb_flow_mrec* in, unsigned long long n, fb_flow_rec* out, unsigned long long* d_n,
                        void* scratch, hipStream_t s);

// Capture-time pass of a timed context's update (fb_time.hip): after K2, over the same FlowParams
// (its record slots, n_slots of them), brings each touched flow's FlowTime forward; ts = the batch's
// capture timestamps by frame index; scratch: time_scratch_bytes(n_slots, log2(cap)).
uint64_t time_scratch_bytes(uint32_t n_slots, uint32_t cap_bits);
// the scratch's sort input (FlowParams::tkv, written by K2); launch_time_prepare marks every record
// slot "no flow" before K2 (invalid slots and non-SESSION records get no entry)
unsigned long long* time_key_array(void* scratch);
hipError_t launch_time_prepare(void* scratch, uint32_t n_slots, hipStream_t s);
hipError_t launch_time_update(const FlowParams& p, uint32_t n_slots, uint64_t cap, FlowTime* plane,
                              const unsigned long long* ts, void* scratch, hipStream_t s);
hipError_t launch_time_remap(const FlowTime* old, const uint32_t* remap, unsigned long long old_cap, FlowTime* nw,
                             hipStream_t s);
hipError_t launch_time_export(const FlowSlot* table, const FlowTime* plane, unsigned long long cap, fb_flow_time* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s);

// Per-flow history characters of the last update (fb_hist.hip): the update's FlowParams (its
// entries, transposed original rows, combined-group maps, per-slot counts) and the outputs.
// cnt: flow_history_cnt_bytes(chunks) of scratch (hot partitions split over chunk blocks), or null
uint64_t flow_history_cnt_bytes(uint32_t chunks);
hipError_t launch_flow_history(const FlowParams& p, uint32_t chunks, uint32_t* hist_slot, uint8_t* hist,
                               uint32_t* n_hist, uint32_t* slow, uint32_t* cnt, hipStream_t s);

// Enrichment tables (fb_set_asn_tables / fb_set_blacklists, fb_enrich.hip).  Blacklists are
// flattened per family into disjoint elementary intervals: bl*_pos[i] = first address of
// interval i (ascending), bl*_mask[i] = the lists whose ranges cover it; an address takes the
// mask of the last interval starting at or before it (none: 0).
struct EnrichTables {
    const fb_asn_range* asn4;
    const fb_asn_range* asn6;
    const uint32_t* bl4_pos;
    const unsigned long long* bl4_mask;
    const uint4* bl6_pos;  // 4 words, session_key order (word 0 most significant)
    const unsigned long long* bl6_mask;
    uint32_t n4, n6, m4, m6;
};
hipError_t launch_ip_lookup(const EnrichTables& t, const fb_ip* ips, uint32_t n, int32_t* asn,
                            unsigned long long* lists, hipStream_t s);
hipError_t launch_flow_enrich(const EnrichTables& t, const DevConfig* cfg, const FlowSlot* table,
                              unsigned long long cap, uint32_t new_only, uint32_t batch, fb_flow_enrich* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s);

hipError_t launch_dns_parse(const uint8_t* frames, unsigned long long frames_bytes, const fb_dns_out* dns, uint32_t n,
                            const fb_batch_stats* stats, fb_dns_msg* msgs, char* names, fb_ip* addrs, hipStream_t s);

}  // namespace fbk
