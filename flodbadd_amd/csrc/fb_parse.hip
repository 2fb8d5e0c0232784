// fb_parse.hip -- gfx950 parse + classify kernels: k_parse_seg (streaming, per-wavefront
// compaction into 64-frame output segments; also the two passes of the parsed-packet dense path)
// and k_parse_dense (single-pass batch-wide output of a frame batch, decoupled look-back).
//
// One wavefront lane per frame.  Replaces, per frame:
//   parse_packet_pcap                 src/packets.rs:603-802 (pnet_packet 0.35.0 decode)
//   service-port direction + key      src/packets.rs:232-311 (get_name_from_port, port_vulns.rs:213)
//   is_originator                     src/packets.rs:316-319
//   Local/Global session filter       src/packets.rs:321-327, sessions.rs:660-672, ip.rs:199-242
//   PACKET_STATS pre-filter counters  src/packets.rs:211-227
//   map_tcp_flags (history char)      src/packets.rs:561-601
//
// The device functions below (header decode, classification, history char) serve the frame and
// the parsed-packet instances alike.  Loads: four unaligned header loads
// per frame at frame offsets 10, 26, 42 (16 B) and 66 (4 B) so every decoder field sits at a
// fixed dword/byte position; buffer loads are range-checked against frames_bytes, so nothing
// reads past the batch.
#include "fb_internal.h"

namespace fbk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Cache policy (buffer instruction aux bits) of the frame-header loads and the record stores.
// Records are stored `nt` (aux 2): +2-3 % at C2 in interleaved A/B runs.  The header loads stay
// default: the three overlapping 16-B loads of a frame reuse its lines in L1, and `nt` loads
// (which bypass L1) cost 20 %.
#ifndef FB_LD_AUX
#define FB_LD_AUX 0
#endif
#ifndef FB_ST_AUX
#define FB_ST_AUX 2
#endif

__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, FB_LD_AUX);
}

// be16 of bytes 0,1 / 2,3 of a little-endian dword.
__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t w) { return ((w >> 8) & 0xff00u) | (w >> 24); }
__device__ __forceinline__ uint32_t bswap(uint32_t w) { return __builtin_bswap32(w); }

__device__ __forceinline__ uint32_t svc(const uint32_t* bm, uint32_t p) { return (bm[p >> 5] >> (p & 31)) & 1u; }

// map_tcp_flags, src/packets.rs:561-601.
__device__ __forceinline__ uint32_t hist_char(uint32_t fl, uint32_t plen, bool orig) {
    uint32_t c;
    if ((fl & 0x02u) && !(fl & 0x10u)) c = 'S';
    else if ((fl & 0x02u) && (fl & 0x10u)) c = 'H';
    else if (fl & 0x01u) c = 'F';
    else if (fl & 0x04u) c = 'R';
    else if (plen > 0u) c = '>';
    else if (fl & 0x10u) c = 'A';
    else return '-';
    if (c == '>') return orig ? '>' : '<';
    return orig ? c : c + 32u;  // lower-case for the responder
}

// Header window of a frame at offset o.  The decoder wants f[10..57] and f[66..69] as dwords
// (so the IPv4/IPv6/TCP fields sit at fixed dword positions), but frame offsets are arbitrary and
// o + 10 is 2 mod 4 for the usual 4-aligned frames: 16-B loads at such addresses cost ~8 % of a
// load/store stream on MI355X (tools/ubench_align.hip: 3.9 vs 4.2 TB/s).  So the loads are
// dword-aligned at a = (o + 10) & ~3 and the window is realigned in registers (v_alignbyte by
// s = (o + 10) & 3, hdr_view below) when the frame is decoded.
#ifndef FB_HDR_ALIGNED
#define FB_HDR_ALIGNED 1
#endif
struct Hdr {
#if FB_HDR_ALIGNED
    u32x4 A, B, C;   // f[a .. a+48)
    uint32_t E;      // f[a+48 .. a+52)
    uint32_t D0, D1; // f[a+56 .. a+64)  (holds f[66..69])
#else
    u32x4 A, B, C;  // f[10..25] f[26..41] f[42..57]
    uint32_t Dz;    // f[66..69] (IPv6 TCP data offset + flags)
#endif
};

// f[10..57] as A, B, C and f[66..69] as Dz, for the frame at offset o.
__device__ __forceinline__ void hdr_view(const Hdr& h, uint32_t o, u32x4& A, u32x4& B, u32x4& C, uint32_t& Dz) {
#if FB_HDR_ALIGNED
    const uint32_t s = (o + 10u) & 3u;
    auto al = [s](uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbyte(hi, lo, s); };
    A = u32x4{al(h.A.y, h.A.x), al(h.A.z, h.A.y), al(h.A.w, h.A.z), al(h.B.x, h.A.w)};
    B = u32x4{al(h.B.y, h.B.x), al(h.B.z, h.B.y), al(h.B.w, h.B.z), al(h.C.x, h.B.w)};
    C = u32x4{al(h.C.y, h.C.x), al(h.C.z, h.C.y), al(h.C.w, h.C.z), al(h.E, h.C.w)};
    Dz = al(h.D1, h.D0);
#else
    (void)o;
    A = h.A;
    B = h.B;
    C = h.C;
    Dz = h.Dz;
#endif
}

struct Pkt {
    uint32_t cls;         // fb_class after filtering
    uint32_t w[14];       // the fb_pkt_out record (SESSION) / dns fields (DNS)
    bool tcp, v4, bad;    // stats bits (valid when session or filtered)
};

// ---- process_parsed_packet, src/packets.rs:202-327, for one SessionPacketData -------------
// (raw 5-tuple src/dst/ports as parsed, L4 payload length, IP length, TCP flags if any) ->
// canonical session key, originator, local/global filter, history char; k.cls = SESSION or
// FILTERED.  Shared by the frame path (process_frame) and the parsed-packet path.
__device__ __forceinline__ void classify_session(const DevConfig* cfg, const DevConfig* gcfg, uint32_t proto,
                                                 uint32_t fam, const uint32_t (&src)[4], const uint32_t (&dst)[4],
                                                 uint32_t sport, uint32_t dport, uint32_t hasf, uint32_t flags,
                                                 uint32_t plen, uint32_t iplen, uint32_t idx, Pkt& k) {
    const uint32_t* bm = cfg->service_bitmap;
    k.tcp = proto == 6u;
    k.v4 = fam == 2u;
    const uint32_t S = svc(bm, sport), Dsv = svc(bm, dport);
    bool swap;
    if (S && !Dsv) {
        swap = true;
    } else if (S && Dsv) {
        // flags only count for TCP (src/packets.rs:257-275); otherwise the port tiebreak
        const bool tf = hasf && proto == 6u && (flags & 0x02u);
        if (tf && !(flags & 0x10u)) swap = false;       // SYN
        else if (tf && (flags & 0x10u)) swap = true;    // SYN+ACK
        else swap = sport < dport;                      // port tiebreak (smaller port = server)
    } else {
        swap = false;
    }
    // is_originator: raw == key field-wise; with a swap that holds only for src==dst & sport==dport.
    const bool orig = !swap || (src[0] == dst[0] && src[1] == dst[1] && src[2] == dst[2] &&
                                src[3] == dst[3] && sport == dport);
    uint32_t ks[4], kd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ks[j] = swap ? dst[j] : src[j];
        kd[j] = swap ? src[j] : dst[j];
    }
    const uint32_t kport_s = swap ? dport : sport, kport_d = swap ? sport : dport;
    const bool lan_s = fam == 2u ? lan_v4(ks[0]) : lan_v6(cfg, gcfg, ks);
    const bool lan_d = fam == 2u ? lan_v4(kd[0]) : lan_v6(cfg, gcfg, kd);
    uint32_t meta = hasf;
    meta |= swap ? FB_META_SWAP : 0u;
    meta |= orig ? FB_META_ORIGINATOR : 0u;
    meta |= lan_s ? FB_META_LOCAL_SRC : 0u;
    meta |= lan_d ? FB_META_LOCAL_DST : 0u;
    meta |= own_ip(cfg, gcfg, fam, ks) ? FB_META_SELF_SRC : 0u;
    meta |= own_ip(cfg, gcfg, fam, kd) ? FB_META_SELF_DST : 0u;
    meta |= (swap ? S : Dsv) ? FB_META_DST_SERVICE : 0u;  // service(key dst port)
    const uint32_t hc = hasf ? hist_char(flags, plen, orig) : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        k.w[j] = ks[j];
        k.w[4 + j] = kd[j];
    }
    k.w[8] = kport_s | (kport_d << 16);
    k.w[9] = proto | (fam << 8);
    k.w[10] = plen;
    k.w[11] = iplen;
    k.w[12] = flags | (meta << 8) | (hc << 16);
    k.w[13] = idx;
    const bool local = lan_s && lan_d;  // is_local_session! (symmetric in src/dst)
    const uint32_t f = cfg->filter;
    const bool drop = (f == FB_FILTER_LOCAL_ONLY && !local) || (f == FB_FILTER_GLOBAL_ONLY && local);
    k.cls = drop ? FB_CLASS_FILTERED : FB_CLASS_SESSION;
}

// Decode + classify one frame from its header vectors; a field is only used when the pnet
// length rules guarantee it lies inside the frame's caplen.
__device__ __forceinline__ void process_frame(__amdgpu_buffer_rsrc_t r, const DevConfig* cfg,
                                              const DevConfig* gcfg, const Hdr& h, uint32_t o0, uint32_t o1,
                                              uint32_t fbytes, uint32_t idx, Pkt& k) {
    k.cls = FB_CLASS_DROP;
    k.tcp = false;
    k.v4 = false;
    const bool okoff = o1 >= o0 && o1 <= fbytes;
    k.bad = !okoff;
    const uint32_t L = okoff ? o1 - o0 : 0u;
    u32x4 A, B, C;
    uint32_t Dz;
    hdr_view(h, o0, A, B, C, Dz);
    if (L < 14u) return;                       // EthernetPacket::new -> None
    const uint32_t et = be16_hi(A.x);          // f[12..13]
    const uint32_t n = L - 14u;
    uint32_t src[4] = {0u, 0u, 0u, 0u}, dst[4] = {0u, 0u, 0u, 0u};
    uint32_t l4off, l4len, proto, d0, d3, iplen, fam;
    if (et == 0x0800u) {                       // IPv4, src/packets.rs:612-700
        if (n < 20u) return;
        const uint32_t ihl4 = (A.y & 0xfu) * 4u;             // version not checked (pnet)
        const uint32_t tot = be16_hi(A.y);                   // ip[2..3]
        proto = (A.w >> 8) & 0xffu;                          // ip[9]
        const uint32_t start = ihl4 > 20u ? ihl4 : 20u;      // 20 + options
        const uint32_t plen = tot > ihl4 ? tot - ihl4 : 0u;  // sat(total_length - ihl*4)
        l4len = n > start ? min(start + plen, n) - start : 0u;
        l4off = 14u + start;
        src[0] = bswap(B.x);                                 // ip[12..15]
        dst[0] = bswap(B.y);                                 // ip[16..19]
        iplen = tot;
        fam = 2u;
        if (start == 20u) {
            d0 = B.z;                                        // f[34..37]
            d3 = C.y;                                        // f[46..49]
        } else {                                             // IPv4 options: dependent load
            const u32x4 E = ld16(r, o0 + l4off);
            d0 = E.x;
            d3 = E.w;
        }
    } else if (et == 0x86DDu) {                // IPv6, src/packets.rs:701-799
        if (n < 40u) return;
        const uint32_t plen6 = be16_lo(A.z);                 // ip[4..5]
        proto = (A.z >> 16) & 0xffu;                         // ip[6] next header
        src[0] = bswap(A.w); src[1] = bswap(B.x); src[2] = bswap(B.y); src[3] = bswap(B.z);
        dst[0] = bswap(B.w); dst[1] = bswap(C.x); dst[2] = bswap(C.y); dst[3] = bswap(C.z);
        l4off = 54u;
        l4len = n > 40u ? min(40u + plen6, n) - 40u : 0u;
        iplen = plen6 + 40u;
        fam = 10u;
        d0 = C.w;                                            // f[54..57]
        d3 = Dz;                                             // f[66..69]
    } else {
        return;                                              // VLAN, ARP, ... -> None
    }
    uint32_t sport, dport, flags = 0u, hasf = 0u, plen;
    if (proto == 6u) {                         // TcpPacket::new needs 20 bytes
        if (l4len < 20u) return;
        sport = be16_lo(d0);
        dport = be16_hi(d0);
        const uint32_t doff = (d3 & 0xffu) >> 4;
        flags = (d3 >> 8) & 0xffu;
        hasf = 1u;
        const uint32_t hs = doff > 5u ? doff * 4u : 20u;
        plen = l4len <= hs ? 0u : l4len - hs;
        if (sport == 53u || dport == 53u) {    // DNS over TCP, src/packets.rs:638-650
            if (plen < 2u) return;
            k.cls = FB_CLASS_DNS;
            k.w[0] = idx;
            k.w[1] = o0 + l4off + hs + 2u;
            k.w[2] = plen - 2u;
            k.w[3] = 6u | (fam << 8);
            return;
        }
    } else if (proto == 17u) {                 // UdpPacket::new needs 8 bytes
        if (l4len < 8u) return;
        sport = be16_lo(d0);
        dport = be16_hi(d0);
        plen = l4len - 8u;
        if (sport == 53u || dport == 53u) {    // DNS over UDP, src/packets.rs:681-686
            k.cls = FB_CLASS_DNS;
            k.w[0] = idx;
            k.w[1] = o0 + l4off + 8u;
            k.w[2] = plen;
            k.w[3] = 17u | (fam << 8);
            return;
        }
    } else {
        return;
    }

    classify_session(cfg, gcfg, proto, fam, src, dst, sport, dport, hasf, flags, plen, iplen, idx, k);
}

// k_parse_seg instances: kFlagsProduct = the plain segmented output, or one of
constexpr uint32_t kFlagsProduct = 0u;
constexpr uint32_t kPartOut = 8u;     // k_parse_seg: also the flow-table partition of each SESSION
                                      // record slot (P.rec_part), for the update that follows
constexpr uint32_t kCountOnly = 16u;  // dense pass 1: segment counts, classes and stats, no records
constexpr uint32_t kDense = 32u;      // dense pass 2: records / DNS records straight to their
                                      // batch-wide positions (P.pre), no counts, classes or stats


__device__ __forceinline__ void load_headers1(__amdgpu_buffer_rsrc_t rs, uint32_t o, Hdr& h) {
#if FB_HDR_ALIGNED
    const uint32_t a = (o + 10u) & ~3u;
    h.A = ld16(rs, a);
    h.B = ld16(rs, a + 16u);
    h.C = ld16(rs, a + 32u);
    // (E and D as one 16-B load -- one VMEM instruction fewer -- measured 2 % slower on C2 and 1 %
    // on C3, tools/r3_ab_parse.sh)
    h.E = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 48u, 0, FB_LD_AUX);
    const u32x2 d = __builtin_amdgcn_raw_buffer_load_b64(rs, a + 56u, 0, FB_LD_AUX);
    h.D0 = d.x;
    h.D1 = d.y;
#else
    h.A = ld16(rs, o + 10u);
    h.B = ld16(rs, o + 26u);
    h.C = ld16(rs, o + 42u);
    h.Dz = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 66u, 0, FB_LD_AUX);
#endif
}

// s_barrier that drains this wave's LDS traffic only (never vector memory).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ============================================================================================
// k_parse_seg -- streaming parse + classify with per-wavefront compaction (segmented output).
//
// The batch is cut into segments of 64 frames (one wavefront); segment sg owns output bytes
// [sg*3584, (sg+1)*3584) of `out` = 64 record slots.  The wave classifies its 64 frames (one
// lane per frame), compacts the SESSION records with a ballot prefix-sum into LDS and writes
// them, in packet order, to the segment's first n_session slots with coalesced 16-B stores (the
// segment base is 16-B aligned, so no head/tail splits); DNS records (16 B) go to the segment's
// tail, the j-th at byte (sg+1)*3584 - 16*(j+1).  seg[sg] = n_session | n_dns << 16.  No wave
// waits for any other: no look-back, no cross-block prefix -- the kernel streams at the rate of
// its loads and stores.  Consumers (the session-table update, the host wrapper) read the
// segments through seg[].  One launch may cover several batches (fb_parse_classify_seg_batches_dev):
// the waves stream over the concatenation of their segments, each batch with its own frames,
// outputs and stats.  Batch stats: packed per-batch device words, see the end of the kernel.
// ============================================================================================
#ifndef FB_SEG_WAVES
#define FB_SEG_WAVES 8
#endif
#ifndef FB_SEG_BPC
#define FB_SEG_BPC 3
#endif
#ifndef FB_SEG_DEPTH
#define FB_SEG_DEPTH 1
#endif
constexpr int kSegWaves = FB_SEG_WAVES;
constexpr int kSegDepth = FB_SEG_DEPTH;  // segments of header loads in flight per wave
constexpr int kSegThreads = 64 * kSegWaves;
constexpr uint32_t kSegBytes = 64u * 56u;  // one segment of output: 64 record slots

#ifdef FB_SEG_TRACE
// -DFB_SEG_TRACE (never the product): per block (up to kSegTrBlocks) the real-time ticks of its
// start, its waves' last segment loop end (max), its segments, and its end (max)
// (tools/experiments/seg_trace.py)
constexpr uint32_t kSegTrBlocks = 2048u;
__device__ __forceinline__ unsigned long long seg_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define SEGTR(stmt) do { stmt; } while (0)
#else
#define SEGTR(stmt) do { } while (0)
#endif
template <bool PARSED, uint32_t FLAGS = kFlagsProduct, bool MULTI = false>
__global__ __launch_bounds__(kSegThreads, kSegWaves * FB_SEG_BPC / 4) void k_parse_seg(const ParseParams P,
                                                                                      const SegBatches SB) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: segment resources in SGPRs
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t nseg = SB.total_segs;  // segments of all the launch's batches
    const uint32_t nb = MULTI ? SB.count : 1u;
    constexpr uint32_t kAcc = kMaxSegBatches * 10u;
    __shared__ uint4 s_cfg4[sizeof(DevConfig) / 16];
    // a wave's staging area: its segment's compacted records (64 x 56 B), then -- partition-writing
    // instance -- its update entries (64 x 64 B)
    constexpr uint32_t kStageU64 = (FLAGS & kPartOut) ? 64u * 8u : 64u * 7u;
    __shared__ __attribute__((aligned(16))) unsigned long long s_stage[kSegWaves][kStageU64];
    __shared__ uint32_t s_acc[kAcc + 1];  // per batch: block counters (see the stats section); wave arrivals
    const DevConfig* cfg = reinterpret_cast<const DevConfig*>(s_cfg4);
    const unsigned long long lmask = (1ull << lane) - 1ull;
    unsigned long long* stage = s_stage[wave];
    uint32_t a_s = 0u, a_d = 0u, a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u, a_n = 0u;  // wave-uniform
    uint32_t a_k = 0u;  // the batch the counters belong to
    if (tid <= kAcc) s_acc[tid] = 0u;  // published by the prologue barrier
    SEGTR(if (tid == 0u && b < kSegTrBlocks) P.dtrace[4u * b] = seg_now());

    // Batch of global segment g.  A wave visits its segments in increasing order, and so do its
    // header fetches and its offsets loads, so each keeps a monotone cursor (wave-uniform scalar
    // compares against the kernel arguments; single-batch launches compile it away).
    uint32_t k_q = 0u, k_h = 0u, k_s = 0u;
    auto batch_of = [&](uint32_t& k, uint32_t g) {
        if constexpr (MULTI)
            while (k + 1u < nb && g >= SB.b[k + 1u].seg_start) ++k;
        return k;
    };
    auto frames_rsrc = [&](uint32_t k) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)SB.b[k].frames, (short)0, (int)SB.b[k].frames_bytes, 0x00020000);
    };

    // One segment per iteration with the next segment's header loads in flight.  Every store of
    // an iteration is an unconditional buffer store (lanes with nothing to write use an offset
    // past the resource's end, which the hardware drops), so each iteration issues exactly the
    // same VMEM sequence -- headers(next), offsets(next+1), 8 stores -- and the compiler's vmcnt
    // bookkeeping lets the wait for the next headers pass over this iteration's stores.
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t kOob = 0x80000000u;
    const uint32_t stride = G * kSegWaves;
    const __amdgpu_buffer_rsrc_t r_drop = __builtin_amdgcn_make_buffer_rsrc(SB.b[0].seg, (short)0, 0, 0x00020000);
    auto vmov = [](uint32_t x) {
        uint32_t y;
        asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
        return y;
    };
    // Segment hand-out: the block owns the segments b*W + j + k*stride (W waves, j < W, k >= 0),
    // numbered L = k*W + j in address order.  The waves of a CU are not served evenly by the
    // memory pipeline (with a static share per wave the first wave of a block left after ~55 %
    // of the time of its last one), so after a static first two (L = wave, wave + W) each wave
    // takes the block's next L from an LDS counter, one step ahead of use: a wave that is
    // served faster processes more segments, and the block finishes when its work is done, not
    // when its slowest wave is.  A wave's L (hence its segments) still increase monotonically.
    // Across blocks the share stays fixed: in a 20-batch C2 launch the blocks end between 257 and
    // 469 us with equal shares, but dealing the launch in chunks from a device counter (round 5,
    // tools/experiments/seg_dynamic_chunks.diff) evened them out (459-495 us) and ran slower --
    // 42.4 vs 43.2 Gpps, and 24.3 vs 36.9 for one batch per launch: the memory system's total rate
    // is fixed, the blocks left running go faster, and the counter's round trips cost
    // (profiles/r05_seg_trace_static.txt, r05_seg_trace_dynamic.txt, r05_seg_dynamic_ab.txt).
    // One segment of header loads in flight per wave: X.h = headers of the current segment,
    // X.c its offsets, X.q the offsets of the wave's next segment.  After a segment:
    // X.h <- headers of the next segment from X.q, X.c <- X.q (explicit v_mov: no back-edge copy
    // of a pending load), X.q <- offsets of the one after.  Every step issues the same VMEM
    // sequence (4 header loads, 2 offset loads, 8 stores) and the prologue mirrors it with
    // dropped stores, so the compiler's vmcnt waits let the stores pass.  Segments past the
    // launch's end clamp to the last batch's last offset (nothing is read out of bounds; the
    // step that would use them never runs).
    constexpr int D = kSegDepth;
    static_assert(D == 1, "one segment of header loads in flight (dynamic hand-out)");
    __shared__ uint32_t s_next;  // the block's next segment number L to hand out
    auto seg_of = [&](uint32_t L) { return b * kSegWaves + L % kSegWaves + (L / kSegWaves) * stride; };
    auto grab = [&]() {
        uint32_t v = 0u;
        if (lane == 0u) v = __hip_atomic_fetch_add(&s_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_amdgcn_readfirstlane(v);
    };
    struct Set {
        Hdr h;
        uint2 c, q;
        unsigned long long p;  // kDense: batch-wide prefix of the segment whose headers are in h
    };
    Set SS[D];
    uint4 pin[4];
    auto load_q = [&](uint32_t g, uint2& q) {
        // (off[i + 1] taken from the next lane by a DPP wave shift, the last lane's by one scalar
        // load, measured slower: C2 45.2 -> 42.8 Gpps, C3 -1 % -- the scalar load's lgkmcnt wait
        // also waits for the LDS staging traffic)
        const uint32_t k = batch_of(k_q, g);
        const uint32_t i = (g - SB.b[k].seg_start) * 64u + lane, n = SB.b[k].n;
        const uint32_t* off = SB.b[k].offsets;
        q = make_uint2(off[min(i, n)], off[min(i + 1u, n)]);
    };
    auto load_pre = [&](uint32_t g) {  // kDense (one batch): n_session | n_dns << 32 before segment g
        return P.pre[min(g, nseg - 1u)];
    };
    unsigned long long ppre = 0ull;  // kDense, parsed-packet instance: prefix of the loaded segment
    auto fetch = [&](Set& X, uint32_t g_h, uint32_t next_q) {  // X.q holds segment g_h's offsets
        if constexpr ((FLAGS & kDense) != 0u) X.p = load_pre(g_h);
        load_headers1(frames_rsrc(batch_of(k_h, g_h)), X.q.x, X.h);
        X.c = make_uint2(vmov(X.q.x), vmov(X.q.y));
        load_q(next_q, X.q);
    };
    // stores per step: segmented 8 (+1 partition), count-only 2, dense 6
    constexpr int kStores = (FLAGS & kCountOnly) ? 2 : (FLAGS & kDense) ? 6 : ((FLAGS & kPartOut) ? 13 : 8);
    auto dropped_stores = [&]() {
#pragma unroll
        for (int j = 0; j < kStores; ++j) __builtin_amdgcn_raw_buffer_store_b32(0u, r_drop, kOob + 64u * j, 0, 0);
    };
    auto load_parsed = [&](uint32_t sg) {
        if constexpr ((FLAGS & kDense) != 0u) ppre = load_pre(sg);
        // 56-B records are only 8-B aligned at odd indices: byte-offset buffer loads (a uint4
        // dereference there would claim 16-B alignment the data does not have).  The resource
        // covers this segment's records only (base in 64-bit arithmetic): a batch-wide byte range
        // or offset would overflow 32 bits past 76.7M records.
        const uint32_t sc = min(sg, (P.n - 1u) >> 6);  // segments past the end clamp to the last one
        const uint32_t left = P.n - sc * 64u;
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(P.parsed + (size_t)sc * 64u), (short)0, (int)(min(left, 64u) * 56u), 0x00020000);
        const uint32_t o = min(lane, left - 1u) * 56u;
        const u32x4 x0 = __builtin_amdgcn_raw_buffer_load_b128(rp, o, 0, 0);
        const u32x4 x1 = __builtin_amdgcn_raw_buffer_load_b128(rp, o + 16u, 0, 0);
        const u32x4 x2 = __builtin_amdgcn_raw_buffer_load_b128(rp, o + 32u, 0, 0);
        const u32x2 x3 = __builtin_amdgcn_raw_buffer_load_b64(rp, o + 48u, 0, 0);
        pin[0] = make_uint4(x0.x, x0.y, x0.z, x0.w);
        pin[1] = make_uint4(x1.x, x1.y, x1.z, x1.w);
        pin[2] = make_uint4(x2.x, x2.y, x2.z, x2.w);
        pin[3] = make_uint4(x3.x, x3.y, 0u, 0u);
    };
    // Prologue: the configuration loads and the first offsets loads are issued together (the
    // header loads then wait for one round trip, not two), the configuration goes to LDS, and
    // an LDS-only barrier publishes it while the header loads stay in flight.
    uint32_t Lc = wave, Ln = wave + kSegWaves;  // the wave's current and next segment numbers
    uint32_t sg = seg_of(Lc);
    if (tid == 0u) s_next = 2u * kSegWaves;  // published by the prologue barrier
    constexpr uint32_t kCfg16 = kCfgLdsBytes / 16, kCfgIt = (kCfg16 + kSegThreads - 1) / kSegThreads;
    uint4 cfgv[kCfgIt];
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
#pragma unroll
        for (uint32_t it = 0; it < kCfgIt; ++it) cfgv[it] = src[min(tid + it * kSegThreads, kCfg16 - 1u)];
    }
    if constexpr (!PARSED) {
        load_q(sg, SS[0].q);
    } else {
        load_parsed(sg);
    }
#pragma unroll
    for (uint32_t it = 0; it < kCfgIt; ++it)
        if (tid + it * kSegThreads < kCfg16) s_cfg4[tid + it * kSegThreads] = cfgv[it];
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        constexpr uint32_t kLanOff = offsetof(DevConfig, lan_v6) / 16, kOwnOff = offsetof(DevConfig, own) / 16;
        const uint32_t nl = P.cfg->n_lan_v6 * (sizeof(LanV6) / 16), no = P.cfg->n_own * (sizeof(fb_ip) / 16);
        for (uint32_t k = tid; k < nl; k += kSegThreads) s_cfg4[kLanOff + k] = src[kLanOff + k];
        for (uint32_t k = tid; k < no; k += kSegThreads) s_cfg4[kOwnOff + k] = src[kOwnOff + k];
        // other parity's word, for the next launch (pass 2 of a dense call is not a launch of its own)
        if (b == 0u && tid == 0u && !(FLAGS & kDense)) *P.error_next = 0u;
    }
    if constexpr (!PARSED) fetch(SS[0], sg, seg_of(Ln));
    dropped_stores();
    lds_barrier();  // configuration in LDS (LDS-only barrier: the header loads stay in flight)
    // a wave's counters go to LDS whenever its segments move on to the next batch
    auto flush = [&]() {
        const uint32_t a_tot = a_s + a_f;
        const uint32_t mine[10] = {a_s, a_f, a_d, a_b, a_t, a_tot - a_t, a_4, a_tot - a_4, a_tot, a_n - a_tot - a_d};
        if (lane < 10u) {
            uint32_t v = 0u;
#pragma unroll
            for (int k = 0; k < 10; ++k) v = lane == (uint32_t)k ? mine[k] : v;
            __hip_atomic_fetch_add(&s_acc[a_k * 10u + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        a_s = a_d = a_f = a_t = a_4 = a_b = a_n = 0u;
    };
    auto step = [&](uint32_t sg, Set& X, uint32_t g_next, uint32_t g_after) {
            const uint32_t k = batch_of(k_s, sg);
            if (MULTI && k != a_k) {
                flush();
                a_k = k;
            }
            const SegBatch& B = SB.b[k];
            const uint32_t ls = sg - B.seg_start;  // the segment within its batch
            const uint32_t i = ls * 64u + lane;
            const bool valid = i < B.n;
            Pkt kk;
            if constexpr (!PARSED) {
                process_frame(frames_rsrc(k), cfg, cfg, X.h, valid ? X.c.x : 1u, valid ? X.c.y : 0u, B.frames_bytes, i,
                              kk);
            } else {
                const uint4 a = pin[0], bb = pin[1], cc = pin[2], d = pin[3];
                const uint32_t src[4] = {a.x, a.y, a.z, a.w}, dst[4] = {bb.x, bb.y, bb.z, bb.w};
                const uint32_t proto = cc.y & 0xffu, fam = (cc.y >> 8) & 0xffu;
                kk.bad = false;
                kk.cls = FB_CLASS_DROP;
                kk.tcp = kk.v4 = false;
                if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                    classify_session(cfg, cfg, proto, fam, src, dst, cc.x & 0xffffu, cc.x >> 16, (d.x >> 8) & 1u,
                                     d.x & 0xffu, cc.z, cc.w, d.y, kk);
            }
            const bool is_s = valid && kk.cls == FB_CLASS_SESSION;
            const bool is_d = valid && kk.cls == FB_CLASS_DNS;
            const bool is_f = valid && kk.cls == FB_CLASS_FILTERED;
            const bool counted = is_s || is_f;
            const unsigned long long m_sess = __ballot(is_s), m_dns = __ballot(is_d);
            const uint32_t cs = (uint32_t)__popcll(m_sess), cd = (uint32_t)__popcll(m_dns);
            if (is_s && !(FLAGS & kCountOnly)) {
                unsigned long long* dd = stage + (size_t)__popcll(m_sess & lmask) * 7;
    #pragma unroll
                for (int w = 0; w < 7; ++w)
                    dd[w] = (unsigned long long)kk.w[2 * w] | ((unsigned long long)kk.w[2 * w + 1] << 32);
            }
            __builtin_amdgcn_wave_barrier();
            unsigned long long pw = 0ull;  // kDense: this segment's prefix
            if constexpr ((FLAGS & kDense) != 0u) pw = PARSED ? ppre : X.p;
            // prefetch: headers of this set's next segment (offsets already here), offsets of the
            // one after
            if constexpr (!PARSED) fetch(X, g_next, g_after);
            else load_parsed(g_next);
            if constexpr ((FLAGS & kCountOnly) != 0u) {
                // dense pass 1: the count word and the class only
                const __amdgpu_buffer_rsrc_t r_seg =
                    __builtin_amdgcn_make_buffer_rsrc(B.seg, (short)0, (int)(((B.n + 63u) / 64u) * 4u), 0x00020000);
                const __amdgpu_buffer_rsrc_t r_cls =
                    __builtin_amdgcn_make_buffer_rsrc(B.cls, (short)0, B.cls ? (int)B.n : 0, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b32(cs | (cd << 16), r_seg, lane == 0u ? ls * 4u : kOob, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)kk.cls, r_cls, valid ? i : kOob, 0, 0);
            } else if constexpr ((FLAGS & kDense) != 0u) {
                // dense pass 2: the segment's records at record pw_s of the batch (56 pw_s is 16-B
                // aligned when pw_s is even; otherwise its first 8-B word goes alone and the 16-B
                // body stays aligned), its DNS records at pw_d
                const uint32_t bs = (uint32_t)pw, bd = (uint32_t)(pw >> 32);
                const uint32_t words = cs * 7u, head = cs ? (bs & 1u) : 0u, body = (words - head) >> 1;
                const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<uint8_t*>(P.dense_out) + (size_t)bs * 56u, (short)0, P.dense_out ? (int)(words * 8u) : 0,
                    0x00020000);
                const __amdgpu_buffer_rsrc_t r_dns = __builtin_amdgcn_make_buffer_rsrc(
                    P.dense_dns + bd, (short)0, P.dense_dns ? (int)(cd * 16u) : 0, 0x00020000);
        #pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t cc = lane + 64u * j;
                    const uint32_t src = head + 2u * min(cc, 223u - head);
                    const unsigned long long x = stage[src], y = stage[src + 1u];
                    const u32x4 v = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b128(v, r_out, cc < body ? head * 8u + cc * 16u : kOob, 0, FB_ST_AUX);
                }
                {   // lane 0: the head word (odd base), lane 1: the tail word (odd body remainder)
                    const bool h1 = head && lane == 0u, t1 = ((words - head) & 1u) && lane == 1u;
                    const uint32_t w = lane == 0u ? 0u : (words ? words - 1u : 0u);
                    const unsigned long long x = stage[w];
                    const u32x2 v = {(uint32_t)x, (uint32_t)(x >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b64(v, r_out, (h1 || t1) ? w * 8u : kOob, 0, FB_ST_AUX);
                }
                {
                    const u32x4 v = {kk.w[0], kk.w[1], kk.w[2], kk.w[3]};
                    __builtin_amdgcn_raw_buffer_store_b128(v, r_dns, is_d ? 16u * (uint32_t)__popcll(m_dns & lmask) : kOob,
                                                           0, 0);
                }
            } else {
            // stores: 4 x 16 B of session records, the 8-B tail, one DNS record, the count, the class
                const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<uint8_t*>(B.out) + (size_t)ls * kSegBytes, (short)0, (int)kSegBytes, 0x00020000);
                // the SESSION records (not stored when the fused call's table is the only output)
                const __amdgpu_buffer_rsrc_t r_rec = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<uint8_t*>(B.out) + (size_t)ls * kSegBytes, (short)0,
                    ((FLAGS & kPartOut) != 0u && P.no_records) ? 0 : (int)kSegBytes, 0x00020000);
                const __amdgpu_buffer_rsrc_t r_seg =
                    __builtin_amdgcn_make_buffer_rsrc(B.seg, (short)0, (int)(((B.n + 63u) / 64u) * 4u), 0x00020000);
                const __amdgpu_buffer_rsrc_t r_cls =
                    __builtin_amdgcn_make_buffer_rsrc(B.cls, (short)0, B.cls ? (int)B.n : 0, 0x00020000);
                const uint32_t words = cs * 7u, body = words >> 1;
        #pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t cc = lane + 64u * j;
                    const uint32_t src = min(cc, 223u);
                    const unsigned long long x = stage[2u * src], y = stage[2u * src + 1u];
                    const u32x4 v = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b128(v, r_rec, cc < body ? cc * 16u : kOob, 0, FB_ST_AUX);
                }
                {
                    const bool tail = (words & 1u) && lane == 0u;
                    const unsigned long long x = stage[words ? words - 1u : 0u];
                    const u32x2 v = {(uint32_t)x, (uint32_t)(x >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b64(v, r_rec, tail ? (words - 1u) * 8u : kOob, 0, FB_ST_AUX);
                }
                {
                    const u32x4 v = {kk.w[0], kk.w[1], kk.w[2], kk.w[3]};
                    __builtin_amdgcn_raw_buffer_store_b128(
                        v, r_out, is_d ? kSegBytes - 16u * (1u + (uint32_t)__popcll(m_dns & lmask)) : kOob, 0, 0);
                }
                __builtin_amdgcn_raw_buffer_store_b32(cs | (cd << 16), r_seg, lane == 0u ? ls * 4u : kOob, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)kk.cls, r_cls, valid ? i : kOob, 0, 0);
                if constexpr ((FLAGS & kPartOut) != 0u) {  // the record slot's table partition (K1's histogram)
                    const __amdgpu_buffer_rsrc_t r_part = __builtin_amdgcn_make_buffer_rsrc(
                        P.rec_part + (size_t)ls * 64u, (short)0, 256, 0x00020000);
                    const uint32_t key[10] = {kk.w[0], kk.w[1], kk.w[2], kk.w[3], kk.w[4],
                                              kk.w[5], kk.w[6], kk.w[7], kk.w[8], kk.w[9] & 0xFFFFu};
                    // update entries (UpdEnt, fb_internal.h): 32-B units, two for an IPv6 key, in
                    // the order of their table partition inside the segment -- so the 3-4 entries of
                    // a 128-B line belong to partitions a few hundred apart, which K2 workgroups
                    // running at the same time read (the line is fetched once; in packet order each
                    // entry's line was a line of its own for K2) -- staged in LDS (the records' reads
                    // of the stage come first in this wave's program order) and stored as whole lines
                    const uint32_t rank = (uint32_t)__popcll(m_sess & lmask);
                    const bool v6 = upd_ent_v6(kk.w[9]);
                    const unsigned long long m_v6 = __ballot(is_s && v6);
                    const uint32_t units = cs + (uint32_t)__popcll(m_v6);
                    const uint32_t part = part_of(flow_hash_words(key), P.part_shift);
                    // bitonic sort of (partition | lane) over the wave, non-session lanes last
                    uint32_t sv = (is_s ? part : 0x10000u) << 6 | lane;  // (partitions < 2^16)
#pragma unroll
                    for (uint32_t k = 2; k <= 64u; k <<= 1) {
#pragma unroll
                        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                            const uint32_t o = (uint32_t)__shfl_xor((int)sv, (int)j, 64);
                            const bool up = (lane & k) == 0u, lower = (lane & j) == 0u;
                            sv = (lower == up) ? min(sv, o) : max(sv, o);
                        }
                    }
                    // sorted position i holds lane src: its units start at the sum of the sizes before it
                    const uint32_t src = sv & 63u;
                    const uint32_t sz = lane < cs ? ((m_v6 >> src) & 1ull ? 2u : 1u) : 0u;
                    uint32_t pre = sz;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const uint32_t y = (uint32_t)__shfl_up((int)pre, o, 64);
                        if (lane >= (uint32_t)o) pre += y;
                    }
                    // back to the entry's own lane (forward permute: lane i sends to lane src)
                    const uint32_t uoff = (uint32_t)__builtin_amdgcn_ds_permute((int)(src * 4u), (int)(pre - sz));
                    // partition | unit offset << 16 | IPv6 << 23 (kRec*, fb_internal.h)
                    const uint32_t pw = part | uoff << kRecUnitShift | (v6 ? kRecV6 : 0u);
                    __builtin_amdgcn_raw_buffer_store_b32(pw, r_part, is_s ? rank * 4u : kOob, 0, 0);
                    if (is_s) {
                        const uint32_t meta = (kk.w[12] >> 8) & 0xFFu;
                        const uint32_t hinfo = ((kk.w[12] >> 16) & 0xFFu) | ((kk.w[12] & 0xFFu) << 8) |
                                               ((meta & FB_META_HAS_FLAGS) ? 1u << 16 : 0u) | ((meta >> 3) & 0x1Fu) << 20;
                        const uint32_t aw = kk.w[9] | ((meta & FB_META_ORIGINATOR) ? 1u << 16 : 0u);
                        u32x4* e = reinterpret_cast<u32x4*>(stage + (size_t)uoff * 4u);
                        e[0] = u32x4{kk.w[0], kk.w[4], kk.w[8], aw};
                        e[1] = u32x4{kk.w[10], kk.w[11], kk.w[13], hinfo | rank << 26};
                        if (v6) {
                            e[2] = u32x4{kk.w[1], kk.w[2], kk.w[3], kk.w[5]};
                            e[3] = u32x4{kk.w[6], kk.w[7], 0u, 0u};
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    const __amdgpu_buffer_rsrc_t r_ent = __builtin_amdgcn_make_buffer_rsrc(
                        P.rec_ent + (size_t)ls * 64u * kUpdEntU4, (short)0, (int)(units * 32u), 0x00020000);
#pragma unroll
                    for (uint32_t k = 0; k < kUpdEntU4; ++k) {  // 4 x 1 KB: up to 128 units
                        const uint32_t q = k * 64u + lane;
                        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + (size_t)min(q, 255u) * 2u);
                        __builtin_amdgcn_raw_buffer_store_b128(v, r_ent, q * 16u, 0, 0);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();  // stage reads of this segment before the next writes
            a_s += cs;
            a_d += cd;
            a_f += __popcll(__ballot(is_f));
            a_t += __popcll(__ballot(counted && kk.tcp));
            a_4 += __popcll(__ballot(counted && kk.v4));
            a_b += __popcll(__ballot(valid && kk.bad));
            a_n += __popcll(__ballot(valid));
    };
#ifdef FB_SEG_TRACE
    uint32_t steps_ = 0u;
#endif
    while (sg < nseg) {
        const uint32_t La = grab();
        const uint32_t g_next = seg_of(Ln);
        step(sg, SS[0], g_next, seg_of(La));
        Lc = Ln;
        Ln = La;
        sg = g_next;
        SEGTR(++steps_);
    }
    SEGTR(if (lane == 0u && b < kSegTrBlocks) {
        atomicMax(P.dtrace + 4u * b + 1u, seg_now());
        atomicAdd(P.dtrace + 4u * b + 2u, (unsigned long long)steps_);
    });
    if constexpr ((FLAGS & kDense) != 0u) return;  // pass 1 of the dense call published the stats
    // ---- batch stats, no barrier and no partials read-back:
    // every wave adds its counters into LDS (per batch); the block's last wave (LDS arrival
    // count) adds the block's counters of every batch into that batch's 5 packed device words
    // [ticket:10 | hi:27 | lo:27] (one atomic per word, lane t takes word t % 5 of batch t / 5);
    // the block whose add brings a word's ticket to G owns that word's final totals (old + its
    // own add), writes those two stats fields and zeroes the word for the next launch.  The
    // derived counts (total, udp, ipv6, drop) are linear, so they are counted per wave and summed
    // like the others.
    {
        flush();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t arrived = 0u;
        if (lane == 0u) arrived = __hip_atomic_fetch_add(&s_acc[kAcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        arrived = __shfl(arrived, 0, 64);
        if (arrived == (uint32_t)kSegWaves - 1u) {
            asm volatile("" ::: "memory");
            for (uint32_t t = lane; t < 5u * nb; t += 64u) {
                const uint32_t k = t / 5u, j = t - 5u * k;
                const unsigned long long lo = s_acc[k * 10u + 2u * j], hi = s_acc[k * 10u + 2u * j + 1u];
                unsigned long long* word = P.tick + k * 8u + j;
                const unsigned long long add = (1ull << 54) | (hi << 27) | lo;
                const unsigned long long old = __hip_atomic_fetch_add(word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((old >> 54) != (unsigned long long)G - 1u) continue;
                const unsigned long long tot = old + add, m27 = (1ull << 27) - 1ull;
                const unsigned long long f_lo = tot & m27, f_hi = (tot >> 27) & m27;
                __hip_atomic_store(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fb_batch_stats* S = SB.b[k].stats;
                if (!S) continue;
                if (j == 0u) {
                    S->n_session = f_lo;
                    S->n_filtered = f_hi;
                    S->new_sessions = 0ull;
                    S->updated_sessions = 0ull;
                    S->error = __hip_atomic_load(P.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    S->reserved[0] = S->reserved[1] = S->reserved[2] = 0ull;
                } else if (j == 1u) {
                    S->n_dns = f_lo;
                    S->bad_offsets = f_hi;
                } else if (j == 2u) {
                    S->tcp_processed = f_lo;
                    S->udp_processed = f_hi;
                } else if (j == 3u) {
                    S->ipv4_processed = f_lo;
                    S->ipv6_processed = f_hi;
                } else {
                    S->total_processed = f_lo;
                    S->n_drop = f_hi;
                }
            }
        }
    }
    SEGTR(if (lane == 0u && b < kSegTrBlocks) atomicMax(P.dtrace + 4u * b + 3u, seg_now()));
}

// ============================================================================================
// k_parse_dense -- single-pass batch-wide (dense) output of one frame batch.
//
// Tiles of kDnTileSegs 64-frame segments; block b owns tiles b, b + G, b + 2G ... (G = grid).
// A block is kDnWaves PARSE waves and one STORE wave:
//   parse waves  stream over the block's segments the way k_parse_seg does (one segment per step,
//                the next segment's headers in flight, segments handed out inside the block from
//                an LDS counter), put each segment's compacted SESSION records (from the front)
//                and DNS records (from the back) into the segment's 3,584-B slot of its tile's LDS
//                buffer, store the classes, and count the segment done.  kDnBufs tile buffers: a wave
//                runs up to one tile ahead of the stores.
//   store wave   per tile, in order: waits until the tile's segments are done, publishes the
//                tile's (n_session, n_dns) in an epoch-tagged status word, looks back over its
//                predecessors' words for the tile's batch-wide offset (decoupled look-back, a
//                64-tile window per step), publishes the inclusive prefix, copies the records and
//                DNS records from LDS to their final positions (16-B stores) and frees the buffer.
// No parse wave waits on a look-back: the status-word round trips (~3 us each under streaming
// load, MI355X_MICROARCH.md handoff rows) overlap the parse of the next tile.  Round 2's kernel
// kept the records in registers and ran the look-back and the stores between two block barriers
// (38.5 us per 1M-frame C2 batch, ~8.5 us of it look-back round trips, ~8 us barriers).
//
// Forward progress without assuming every workgroup is resident (a GPU shared with other work
// may not run all of them at once -- the failure round 1's look-back kernel had): a
// look-back that has waited P.steal_polls polls for a predecessor's word computes that tile's
// sums itself (count-only classification of its frames, the same deterministic result the owner
// will publish), CASes them in as the tile's aggregate if the word is still unpublished, and
// walks on.  So a look-back never depends on a workgroup that is not running; in the normal case
// nothing is recomputed.  Inside a block the parse and store waves depend only on each other
// (all resident): a parse wave waits for a buffer only until the store wave has copied the tile
// kDnBufs rounds back, and the store wave waits for segments that parse waves grabbed earlier.
// Geometry measured (C2 / C3 per 1M frames): 16-segment tiles, two buffers, one 15 + 1-wave block
// per CU 37.3-38.4 / 47.9-49.1 us; 20-segment tiles 38.2-38.5 / 50.9; 12 x 3 buffers 41.1-41.5;
// 8 x 3 or 4 buffers 47.9-49.8; poll sleeps of 4 / 16 within noise -- the tile count, not the
// buffering depth, sets the pace.
// ============================================================================================
#ifndef FB_DN_WAVES
#define FB_DN_WAVES 15
#endif
#ifndef FB_DN_TILE
#define FB_DN_TILE 16
#endif
#ifndef FB_DN_BPC
#define FB_DN_BPC 1
#endif
#ifndef FB_DN_LB
#define FB_DN_LB 1
#endif
#ifndef FB_DN_BUFS
#define FB_DN_BUFS 2
#endif
#ifndef FB_DN_SLEEP
#define FB_DN_SLEEP 1
#endif
constexpr int kDnWaves = FB_DN_WAVES;         // parse waves per block (+ the store wave)
constexpr uint32_t kDnTileSegs = FB_DN_TILE;  // segments per tile
constexpr int kDnThreads = 64 * (kDnWaves + 1);
constexpr int kDnLb = FB_DN_LB;  // look-back: status words per lane per step
constexpr uint32_t kDnBufs = FB_DN_BUFS;  // tile buffers: a wave runs up to kDnBufs - 1 tiles ahead of the copies
constexpr uint32_t kDnSlotU64 = kSegBytes / 8u;  // one segment's slot in a tile buffer (448 u64)
static_assert(kDnTileSegs <= 64u, "the store wave holds one segment count per lane");
// tile status word [epoch:8 | P:1 | A:1 | n_dns:27 | n_session:27]: A = the tile's own sums are
// published, P = its inclusive prefix is (k_seg_scan's format)
constexpr unsigned long long kDnA = 1ull << 54, kDnP = 1ull << 55, kDn27 = (1ull << 27) - 1ull;
__device__ __forceinline__ unsigned long long dn_word(uint32_t ep, unsigned long long flag, unsigned long long pair) {
    return ((unsigned long long)ep << 56) | flag | (pair & kDn27) | (((pair >> 32) & kDn27) << 27);
}
__device__ __forceinline__ unsigned long long dn_pair(unsigned long long w) {
    return (w & kDn27) | (((w >> 27) & kDn27) << 32);
}
#ifdef FB_DN_TRACE
// -DFB_DN_TRACE (never the product): per tile t the real-time ticks (100 MHz) when the store wave saw
// it written, published its offset, and when its last slot was copied out; per block its start,
// the end of its parse waves' segment loops (max) and its end (max).  Words: [tile 4 x kDnTrTiles |
// block 4 x kDnTrBlocks] (tools/experiments/dense_trace.py).
constexpr uint32_t kDnTrTiles = 8192u, kDnTrBlocks = 1024u;
__device__ __forceinline__ unsigned long long dn_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define DNTR(stmt) do { stmt; } while (0)
#else
#define DNTR(stmt) do { } while (0)
#endif
struct DnLds {
    unsigned long long buf[kDnBufs][kDnTileSegs][kDnSlotU64];  // tile buffers, one slot per segment
    unsigned long long base[kDnBufs];                     // the buffer's tile: batch-wide offset (pair)
    uint32_t cnt[kDnBufs][kDnTileSegs];                   // per slot n_session | n_dns << 16
    uint32_t pre[kDnBufs][kDnTileSegs];                   // per slot: records | DNS records before it in the tile
    uint32_t done[kDnBufs];                               // slots of the buffer's tile written
    uint32_t copied[kDnBufs];                             // slots of the buffer's tile copied out
    uint32_t ready_round[kDnBufs];                        // the round whose offset base / pre hold
    uint32_t free_round[kDnBufs];                         // the block round the buffer is free for
    uint32_t next;                                        // the next segment number to hand out
    uint32_t acc[11];                                     // the block's stats counters; wave arrivals
};

// Blocks per CU: FB_DN_BPC (default one 16-wave block: 15 parse + 1 store, two 57-KiB tile
// buffers).  The host caps the occupancy query at FB_DN_BPC: with 9-wave blocks (8 + 1) at 95 VGPRs
// the query said two per CU but the hardware admitted one (each block puts three waves on one SIMD;
// two blocks there need six, the VGPRs allow five), and the grid's second half ran only after the
// first: the look-backs of the resident half waited for it (5.8 ms per C2 batch).
__global__ __launch_bounds__(kDnThreads, (FB_DN_BPC * kDnThreads + 255) / 256) void k_parse_dense(const ParseParams P,
                                                                                        const SegBatch B) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t nt = P.ntiles, ep = P.dep, n = B.n;
    const uint32_t nseg = (n + 63u) / 64u;
    __shared__ uint4 s_cfg4[sizeof(DevConfig) / 16];
    __shared__ DnLds L;
    const DevConfig* cfg = reinterpret_cast<const DevConfig*>(s_cfg4);
    const unsigned long long lmask = (1ull << lane) - 1ull;
    constexpr uint32_t kOob = 0x80000000u;
    const __amdgpu_buffer_rsrc_t r_fr =
        __builtin_amdgcn_make_buffer_rsrc((void*)B.frames, (short)0, (int)B.frames_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_cls = __builtin_amdgcn_make_buffer_rsrc(B.cls, (short)0, B.cls ? (int)n : 0, 0x00020000);
    const bool parser = wave < (uint32_t)kDnWaves;
    if (tid < kDnBufs) {
        L.done[tid] = 0u;
        L.copied[tid] = 0u;
        L.ready_round[tid] = ~0u;
        L.free_round[tid] = tid;
    }
    if (tid <= 10u) L.acc[tid] = 0u;
    if (tid == 0u) L.next = 2u * kDnWaves;  // the first two segments of each wave are static
    DNTR(if (tid == 0u && b < kDnTrBlocks) P.dtrace[4u * kDnTrTiles + 4u * b] = dn_now());

    // block-local segment number Ls -> global segment: round Ls / T of the block (tile b + round G),
    // slot Ls % T of the tile
    auto seg_of = [&](uint32_t Ls) { return (b + (Ls / kDnTileSegs) * G) * kDnTileSegs + Ls % kDnTileSegs; };
    auto grab = [&]() {
        uint32_t v = 0u;
        if (lane == 0u) v = __hip_atomic_fetch_add(&L.next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_amdgcn_readfirstlane(v);
    };
    auto load_q = [&](uint32_t g, uint2& q) {  // frame offsets of segment g (past the end: clamped)
        const uint32_t i = min(g, nseg) * 64u + lane;
        q = make_uint2(B.offsets[min(i, n)], B.offsets[min(i + 1u, n)]);
    };
    auto vmov = [](uint32_t x) {
        uint32_t y;
        asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
        return y;
    };
    // parse waves: the current segment's headers (h) and offsets (c), the next segment's offsets (q)
    Hdr h;
    uint2 c = make_uint2(0u, 0u), q = make_uint2(0u, 0u);
    uint32_t Lc = wave, Ln = wave + kDnWaves;
    if (parser) load_q(seg_of(Lc), q);  // in flight with the configuration copy
    {
        constexpr uint32_t kCfg16 = kCfgLdsBytes / 16;
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        for (uint32_t k = tid; k < kCfg16; k += kDnThreads) s_cfg4[k] = src[k];
        constexpr uint32_t kLanOff = offsetof(DevConfig, lan_v6) / 16, kOwnOff = offsetof(DevConfig, own) / 16;
        const uint32_t nl = P.cfg->n_lan_v6 * (sizeof(LanV6) / 16), no = P.cfg->n_own * (sizeof(fb_ip) / 16);
        for (uint32_t k = tid; k < nl; k += kDnThreads) s_cfg4[kLanOff + k] = src[kLanOff + k];
        for (uint32_t k = tid; k < no; k += kDnThreads) s_cfg4[kOwnOff + k] = src[kOwnOff + k];
        if (b == 0u && tid == 0u) *P.error_next = 0u;
    }
    auto fetch = [&](uint32_t g_after) {  // q holds the next segment's offsets
        load_headers1(r_fr, q.x, h);
        c = make_uint2(vmov(q.x), vmov(q.y));
        load_q(g_after, q);
    };
    if (parser) {
        fetch(seg_of(Ln));
        __builtin_amdgcn_raw_buffer_store_b8(0u, r_cls, kOob, 0, 0);  // the step's VMEM sequence (dropped store)
    }
    lds_barrier();  // configuration and block state in LDS (loads stay in flight); the last block barrier

    if (!parser) {
        // ---------------- store wave: the tiles' offsets ----------------
        // (n_session, n_dns) of tile j, computed by this wave (the look-back's fallback)
        auto tile_pair = [&](uint32_t j) {
            unsigned long long acc = 0ull;
            for (uint32_t sgi = 0; sgi < kDnTileSegs; ++sgi) {
                const uint32_t i = (j * kDnTileSegs + sgi) * 64u + lane;
                const bool valid = i < n;
                const uint2 qq = make_uint2(B.offsets[min(i, n)], B.offsets[min(i + 1u, n)]);
                Hdr hh;
                load_headers1(r_fr, qq.x, hh);
                Pkt k;
                process_frame(r_fr, cfg, cfg, hh, valid ? qq.x : 1u, valid ? qq.y : 0u, B.frames_bytes, i, k);
                acc += (unsigned long long)__popcll(__ballot(valid && k.cls == FB_CLASS_SESSION)) |
                       ((unsigned long long)__popcll(__ballot(valid && k.cls == FB_CLASS_DNS)) << 32);
            }
            return acc;
        };
        for (uint32_t r = 0;; ++r) {
            const uint32_t t = b + r * G;
            if (t >= nt) break;
            const uint32_t p = r % kDnBufs;
            const uint32_t segs = min(kDnTileSegs, nseg - t * kDnTileSegs);
            // the buffer serves this round (its previous tile is copied out: done was reset before
            // free_round moved on) and every slot of the tile is written
            while (__hip_atomic_load(&L.free_round[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != r ||
                   __hip_atomic_load(&L.done[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != segs)
                __builtin_amdgcn_s_sleep(FB_DN_SLEEP);
            DNTR(if (lane == 0u && t < kDnTrTiles) P.dtrace[4u * t] = dn_now());
            // per slot exclusive prefixes inside the tile (lane j: slot j), and the tile's sums
            const uint32_t cw = lane < segs ? L.cnt[p][lane] : 0u;
            uint32_t incl = cw;  // n_session | n_dns << 16 never carries (<= 64 per slot, 16 slots)
#pragma unroll
            for (int o = 1; o < (int)kDnTileSegs; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= (uint32_t)o) incl += y;
            }
            if (lane < kDnTileSegs) L.pre[p][lane] = incl - cw;
            const uint32_t tot = __shfl(incl, (int)kDnTileSegs - 1, 64);
            const unsigned long long agg = (unsigned long long)(tot & 0xFFFFu) | ((unsigned long long)(tot >> 16) << 32);
            unsigned long long excl = 0ull;
            if (t == 0u) {
                if (lane == 0u) __hip_atomic_store(P.dstatus, dn_word(ep, kDnP, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (lane == 0u)
                    __hip_atomic_store(P.dstatus + t, dn_word(ep, kDnA, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // window of 64 x kDnLb tiles per step (lane l holds tiles jt-1-(l*kDnLb+k), k < kDnLb:
                // a round's G tiles finish together, so the walk from the last tiles of a round back
                // to the previous round's inclusive prefixes is G tiles long -- one step when
                // 64 kDnLb >= G).  A step waits only for the words in front of the nearest published
                // inclusive prefix (P) it can see, re-polling only those, and walks on when there is
                // none.
                int64_t jt = (int64_t)t;
                auto ready = [&](unsigned long long x) { return (uint32_t)(x >> 56) == ep && (x & (kDnA | kDnP)); };
                auto probe = [&](int k) {
                    const int64_t idx = jt - 1 - (int64_t)(lane * (uint32_t)kDnLb + (uint32_t)k);
                    return idx >= 0 ? __hip_atomic_load(P.dstatus + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : dn_word(ep, kDnP, 0ull);
                };
                for (;;) {
                    unsigned long long v[kDnLb];
#pragma unroll
                    for (int k = 0; k < kDnLb; ++k) v[k] = probe(k);
                    uint32_t sl = 64u, kp = 0u;  // the nearest P: its lane and word (sl 64: none)
                    for (uint32_t spins = 0u;; ++spins) {
                        uint32_t kpl = kDnLb;
#pragma unroll
                        for (int k = kDnLb - 1; k >= 0; --k) kpl = (ready(v[k]) && (v[k] & kDnP)) ? (uint32_t)k : kpl;
                        const unsigned long long pm = __ballot(kpl < (uint32_t)kDnLb);
                        sl = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
                        kp = pm ? (uint32_t)__shfl((int)kpl, (int)sl, 64) : 0u;
                        uint32_t need = 0u;  // unpublished words in front of it
#pragma unroll
                        for (int k = 0; k < kDnLb; ++k)
                            need |= ((lane < sl || (lane == sl && (uint32_t)k < kp)) && !ready(v[k])) ? 1u << k : 0u;
                        unsigned long long late = __ballot(need != 0u);
                        if (late == 0ull) break;
                        if (spins >= P.steal_polls) {
                            // the owners of these tiles may not be running: compute their sums here
                            while (late) {
                                const uint32_t l = (uint32_t)__builtin_ctzll(late);
                                late &= late - 1ull;
                                uint32_t nk = (uint32_t)__shfl((int)need, (int)l, 64);
                                while (nk) {
                                    const uint32_t kk = (uint32_t)__builtin_ctz(nk);
                                    nk &= nk - 1u;
                                    const uint32_t j = (uint32_t)(jt - 1 - (int64_t)(l * (uint32_t)kDnLb + kk));
                                    const unsigned long long w = dn_word(ep, kDnA, tile_pair(j));
#pragma unroll
                                    for (int k = 0; k < kDnLb; ++k) {
                                        if (lane == l && (uint32_t)k == kk) {
                                            atomicCAS(P.dstatus + j, v[k], w);  // unless the owner published meanwhile
                                            v[k] = w;
                                        }
                                    }
                                }
                            }
                            break;
                        }
                        __builtin_amdgcn_s_sleep(FB_DN_SLEEP);
#pragma unroll
                        for (int k = 0; k < kDnLb; ++k)
                            if (!ready(v[k])) v[k] = probe(k);
                    }
                    unsigned long long part = 0ull;
#pragma unroll
                    for (int k = 0; k < kDnLb; ++k)
                        part += (lane < sl || (lane == sl && (uint32_t)k <= kp)) ? dn_pair(v[k]) : 0ull;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
                    excl += part;
                    if (sl < 64u) break;
                    jt -= 64 * kDnLb;
                }
                if (lane == 0u)
                    __hip_atomic_store(P.dstatus + t, dn_word(ep, kDnP, excl + agg), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            // the offset for the parse waves, which copy their slots out (release: pre and base
            // are visible before the round is marked ready -- with relaxed orders the compiler
            // may put the base store after the flag, and a parse wave copied to a stale offset)
            DNTR(if (lane == 0u && t < kDnTrTiles) P.dtrace[4u * t + 1u] = dn_now());
            if (lane == 0u) {
                // (a fault-injection skew moves the session half only, wrapping inside it)
                L.base[p] = P.dn_skew ? ((excl & ~0xFFFFFFFFull) | ((excl + P.dn_skew) & 0xFFFFFFFFull)) : excl;
                __hip_atomic_store(&L.ready_round[p], r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        return;
    }

    // ---------------- parse waves ----------------
    // A written slot stays pending in its wave until the store wave has published its tile's
    // offset; the wave copies it out at a later step.  Two rules keep every wait finite: a wave
    // only blocks on a copy when each slot it holds is written (its tile can then complete without
    // it), and while it waits for a free buffer it copies whatever of its own has become ready (a
    // buffer is free once every slot of its tile kDnBufs rounds back is copied).  At most two pending
    // slots per wave.
    uint32_t a_s = 0u, a_d = 0u, a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u, a_n = 0u;  // wave-uniform
    uint32_t pend0 = ~0u, pend1 = ~0u;  // pending slots' segment numbers Ls, oldest first (~0u: none)
    auto ready_of = [&](uint32_t Ls) {
        const uint32_t rnd = Ls / kDnTileSegs;
        return __hip_atomic_load(&L.ready_round[rnd % kDnBufs], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == rnd;
    };
    auto copy_out = [&](uint32_t Ls) {  // (the tile's offset is published)
        const uint32_t rnd = Ls / kDnTileSegs, p = rnd % kDnBufs, j = Ls % kDnTileSegs;
        const unsigned long long* stage = L.buf[p][j];
        const uint32_t cw = L.cnt[p][j], pw = L.pre[p][j];
        const unsigned long long bp = L.base[p];
        const uint32_t cs = cw & 0xFFFFu, cd = cw >> 16;
        // records at batch-wide record bs (56 bs is 16-B aligned when bs is even; otherwise the
        // first 8-B word goes alone and the 16-B body stays aligned), DNS records at bd.  The buffer
        // resources are based at the slot's destination, so their range check only covers the slot's
        // own records: a destination past the batch's n records (the caller's buffers hold n) would
        // be written outside them.  That needs a corrupted tile offset -- round 4's no-look-back
        // ablation added the real prefix to a fixed one and faulted here -- and drops the slot with
        // error bit 32 instead (checked in 64 bits: a bad offset must not wrap into range).
        const unsigned long long bs64 = (bp & 0xFFFFFFFFull) + (pw & 0xFFFFu), bd64 = (bp >> 32) + (pw >> 16);
        const bool in_range = bs64 + cs <= (unsigned long long)n && bd64 + cd <= (unsigned long long)n;
        if (!in_range && lane == 0u) {  // (the returned value is waited for: the bit is in L2 before this wave
                                        // reports its stats, so the block that writes the batch stats reads it)
            const uint32_t old = __hip_atomic_fetch_or(P.error, 32u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("" ::"v"(old));
        }
        const uint32_t bs = in_range ? (uint32_t)bs64 : 0u, bd = in_range ? (uint32_t)bd64 : 0u;
        const uint32_t words = cs * 7u, head = cs ? (bs & 1u) : 0u, body = (words - head) >> 1;
        const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<uint8_t*>(P.dense_out) + (size_t)bs * 56u, (short)0,
            P.dense_out && in_range ? (int)(words * 8u) : 0, 0x00020000);
        const __amdgpu_buffer_rsrc_t r_dns = __builtin_amdgcn_make_buffer_rsrc(
            P.dense_dns + bd, (short)0, P.dense_dns && in_range ? (int)(cd * 16u) : 0, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t cc = lane + 64u * k;
            const uint32_t src = head + 2u * min(cc, 223u - head);
            const unsigned long long x = stage[src], y = stage[src + 1u];
            const u32x4 v = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
            __builtin_amdgcn_raw_buffer_store_b128(v, r_out, cc < body ? head * 8u + cc * 16u : kOob, 0, FB_ST_AUX);
        }
        {   // lane 0: the head word (odd base), lane 1: the tail word (odd body remainder)
            const bool h1 = head && lane == 0u, t1 = ((words - head) & 1u) && lane == 1u;
            const uint32_t w = lane == 0u ? 0u : (words ? words - 1u : 0u);
            const unsigned long long x = stage[w];
            const u32x2 v = {(uint32_t)x, (uint32_t)(x >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(v, r_out, (h1 || t1) ? w * 8u : kOob, 0, FB_ST_AUX);
        }
        {   // DNS record k of the slot sits at its back, 16 B each
            const unsigned long long* e = stage + kDnSlotU64 - 2u * (min(lane, 63u) + 1u);
            const unsigned long long x = e[0], y = e[1];
            const u32x4 v = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
            __builtin_amdgcn_raw_buffer_store_b128(v, r_dns, lane < cd ? 16u * lane : kOob, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's LDS reads have returned
        if (lane == 0u) {
            const uint32_t t = b + rnd * G, segs = min(kDnTileSegs, nseg - t * kDnTileSegs);
            const uint32_t old = __hip_atomic_fetch_add(&L.copied[p], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old + 1u == segs) {  // the tile's last copy: the buffer serves round rnd + kDnBufs
                DNTR(if (t < kDnTrTiles) P.dtrace[4u * t + 2u] = dn_now());
                L.done[p] = 0u;
                L.copied[p] = 0u;
                __hip_atomic_store(&L.free_round[p], rnd + kDnBufs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    };
    uint32_t sg = seg_of(Lc);
    while (sg < nseg) {
        const uint32_t La = grab();
        const uint32_t g_next = seg_of(Ln);
        const uint32_t i = sg * 64u + lane;
        const bool valid = i < n;
        Pkt kk;
        process_frame(r_fr, cfg, cfg, h, valid ? c.x : 1u, valid ? c.y : 0u, B.frames_bytes, i, kk);
        const bool is_s = valid && kk.cls == FB_CLASS_SESSION;
        const bool is_d = valid && kk.cls == FB_CLASS_DNS;
        const bool is_f = valid && kk.cls == FB_CLASS_FILTERED;
        const bool counted = is_s || is_f;
        const unsigned long long m_sess = __ballot(is_s), m_dns = __ballot(is_d);
        const uint32_t cs = (uint32_t)__popcll(m_sess), cd = (uint32_t)__popcll(m_dns);
        fetch(seg_of(La));  // the next segment's headers, the offsets of the one after
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)kk.cls, r_cls, valid ? i : kOob, 0, 0);
        // the segment's slot in its tile's buffer (free once the tile kDnBufs rounds back is copied out);
        // meanwhile this wave's own ready slots go out
        const uint32_t rnd = Lc / kDnTileSegs, p = rnd % kDnBufs, j = Lc % kDnTileSegs;
        for (;;) {
            if (pend0 != ~0u && ready_of(pend0)) {
                copy_out(pend0);
                pend0 = pend1;
                pend1 = ~0u;
            }
            if (__hip_atomic_load(&L.free_round[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == rnd) break;
            __builtin_amdgcn_s_sleep(FB_DN_SLEEP);
        }
        unsigned long long* slot = L.buf[p][j];
        if (is_s) {
            unsigned long long* dd = slot + (size_t)__popcll(m_sess & lmask) * 7;
#pragma unroll
            for (int w = 0; w < 7; ++w)
                dd[w] = (unsigned long long)kk.w[2 * w] | ((unsigned long long)kk.w[2 * w + 1] << 32);
        }
        if (is_d) {
            unsigned long long* dd = slot + kDnSlotU64 - 2u * (1u + (uint32_t)__popcll(m_dns & lmask));
            dd[0] = (unsigned long long)kk.w[0] | ((unsigned long long)kk.w[1] << 32);
            dd[1] = (unsigned long long)kk.w[2] | ((unsigned long long)kk.w[3] << 32);
        }
        if (lane == 0u) L.cnt[p][j] = cs | (cd << 16);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is written before it is counted
        if (lane == 0u) __hip_atomic_fetch_add(&L.done[p], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        // pend this slot; with two already pending, the oldest goes out first (every slot this wave
        // holds is written now, so waiting for its tile cannot wait for this wave)
        if (pend1 != ~0u) {
            while (!ready_of(pend0)) __builtin_amdgcn_s_sleep(FB_DN_SLEEP);
            copy_out(pend0);
            pend0 = pend1;
            pend1 = ~0u;
        }
        if (pend0 == ~0u) pend0 = Lc;
        else pend1 = Lc;
        a_s += cs;
        a_d += cd;
        a_f += __popcll(__ballot(is_f));
        a_t += __popcll(__ballot(counted && kk.tcp));
        a_4 += __popcll(__ballot(counted && kk.v4));
        a_b += __popcll(__ballot(valid && kk.bad));
        a_n += __popcll(__ballot(valid));
        Lc = Ln;
        Ln = La;
        sg = g_next;
    }
    DNTR(if (lane == 0u && b < kDnTrBlocks) atomicMax(P.dtrace + 4u * kDnTrTiles + 4u * b + 1u, dn_now()));
    for (uint32_t k = 0; k < 2u; ++k) {  // the last pending slots
        if (pend0 == ~0u) break;
        while (!ready_of(pend0)) __builtin_amdgcn_s_sleep(FB_DN_SLEEP);
        copy_out(pend0);
        pend0 = pend1;
        pend1 = ~0u;
    }
    DNTR(if (lane == 0u && b < kDnTrBlocks) atomicMax(P.dtrace + 4u * kDnTrTiles + 4u * b + 2u, dn_now()));
    // batch stats: as k_parse_seg (one batch): wave counters into LDS, the block's last parse wave
    // adds the block's into the five packed device words; the block completing a word writes its
    // fields
    {
        const uint32_t a_tot = a_s + a_f;
        const uint32_t mine[10] = {a_s, a_f, a_d, a_b, a_t, a_tot - a_t, a_4, a_tot - a_4, a_tot, a_n - a_tot - a_d};
        if (lane < 10u) {
            uint32_t v = 0u;
#pragma unroll
            for (int k = 0; k < 10; ++k) v = lane == (uint32_t)k ? mine[k] : v;
            __hip_atomic_fetch_add(&L.acc[lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t arrived = 0u;
        if (lane == 0u) arrived = __hip_atomic_fetch_add(&L.acc[10], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        arrived = __shfl(arrived, 0, 64);
        if (arrived == (uint32_t)kDnWaves - 1u && lane < 5u) {
            asm volatile("" ::: "memory");
            const uint32_t j = lane;
            const unsigned long long lo = L.acc[2u * j], hi = L.acc[2u * j + 1u];
            unsigned long long* word = P.tick + j;
            const unsigned long long add = (1ull << 54) | (hi << 27) | lo;
            const unsigned long long old = __hip_atomic_fetch_add(word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((old >> 54) == (unsigned long long)G - 1u) {
                const unsigned long long tot = old + add, m27 = (1ull << 27) - 1ull;
                const unsigned long long f_lo = tot & m27, f_hi = (tot >> 27) & m27;
                __hip_atomic_store(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fb_batch_stats* S = B.stats;
                if (S) {
                    if (j == 0u) {
                        S->n_session = f_lo;
                        S->n_filtered = f_hi;
                        S->new_sessions = 0ull;
                        S->updated_sessions = 0ull;
                        S->error = __hip_atomic_load(P.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        S->reserved[0] = S->reserved[1] = S->reserved[2] = 0ull;
                    } else if (j == 1u) {
                        S->n_dns = f_lo;
                        S->bad_offsets = f_hi;
                    } else if (j == 2u) {
                        S->tcp_processed = f_lo;
                        S->udp_processed = f_hi;
                    } else if (j == 3u) {
                        S->ipv4_processed = f_lo;
                        S->ipv6_processed = f_hi;
                    } else {
                        S->total_processed = f_lo;
                        S->n_drop = f_hi;
                    }
                }
            }
        }
    }
}

hipError_t launch_parse_dense(const ParseParams& p, const SegBatch& b, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(k_parse_dense, dim3(grid), dim3(kDnThreads), 0, s, p, b);
    return hipGetLastError();
}
hipError_t occupancy_parse_dense(int* blocks_per_cu) {
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_parse_dense, kDnThreads, 0);
    if (e == hipSuccess && *blocks_per_cu > FB_DN_BPC) *blocks_per_cu = FB_DN_BPC;  // (the query can overstate it)
    return e;
}
uint32_t parse_dense_tile_segs() { return kDnTileSegs; }

hipError_t launch_parse_seg(const ParseParams& p, const SegBatches& sb, uint32_t grid, hipStream_t s, SegPass pass) {
    const dim3 g(grid), t(kSegThreads);
    if (pass == SegPass::kCount) {
        if (p.parsed) hipLaunchKernelGGL((k_parse_seg<true, kCountOnly>), g, t, 0, s, p, sb);
        else hipLaunchKernelGGL((k_parse_seg<false, kCountOnly>), g, t, 0, s, p, sb);
    } else if (pass == SegPass::kDenseOut) {
        if (p.parsed) hipLaunchKernelGGL((k_parse_seg<true, kDense>), g, t, 0, s, p, sb);
        else hipLaunchKernelGGL((k_parse_seg<false, kDense>), g, t, 0, s, p, sb);
    } else if (p.parsed) {
        hipLaunchKernelGGL((k_parse_seg<true>), g, t, 0, s, p, sb);
    } else if (sb.count > 1u) {
        hipLaunchKernelGGL((k_parse_seg<false, kFlagsProduct, true>), g, t, 0, s, p, sb);
    } else if (p.rec_part) {  // instantiated after the headline instance: its code placement is unchanged
        hipLaunchKernelGGL((k_parse_seg<false, kFlagsProduct | kPartOut>), g, t, 0, s, p, sb);
    } else {
        hipLaunchKernelGGL((k_parse_seg<false>), g, t, 0, s, p, sb);
    }
    return hipGetLastError();
}
hipError_t occupancy_parse_seg(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (k_parse_seg<false>), kSegThreads, 0);
}
uint32_t parse_seg_block_threads() { return kSegThreads; }

// ============================================================================================
// k_parse_seg_queue -- k_parse_seg's segmented output as ONE resident kernel fed batch by batch
// (fb_seg_queue_*).  A single-batch launch pays its prologue (configuration, then the first offsets,
// then the first headers: two dependent round trips before a wave has work) and the tail of the
// batch's last segments on every call: 27.8 us of kernel per 1M-frame C2 batch against 22.4 us per
// batch inside a multi-batch launch (profiles/r05_single_batch_trace.txt).  Here the waves stream
// from one batch into the next as k_parse_seg's multi-batch instance does, but the batches arrive
// while the kernel runs: the host writes batch k into slot k % depth of a ring in pinned host memory
// and then its tail word; a block learns batch k's descriptor once (the first wave that needs it
// copies it from the device side of the ring into the block's LDS, the others wait on the LDS copy;
// one block at a time reads the host's ring over PCIe into the device side) and takes batch k's
// segments in chunks from the slot's device counter, handing them to its waves through an LDS
// counter.  A wave never blocks while it holds unprocessed segments: when the next batch is not
// published yet it drains its pipeline and only then waits.
// Completion without a grid barrier (blocks need not be resident together): each wave, before it
// counts itself done with a batch (LDS arrival per batch), has waited for its own stores; the
// block's last wave adds the block's counters into the batch's stats words (the block completing a
// word writes its stats fields), writes the XCD's L2 back (agent release) and counts the block in
// the batch's device counter; the last block resets that counter and stores k + 1 into the slot's
// completion word in host memory (system release), which fb_seg_queue_query polls.  The host never
// reuses a slot before its batch completed, so per-slot LDS and device state is reset by the batch's
// last user.  A block that waits idle_ticks for a batch, or sees the host's stop word with nothing
// left, leaves; an expired queue reports it in the control block's status word.
// ============================================================================================
// The queue kernel's output stores are write-through (sc1): a batch is complete when the waves that
// wrote it have their stores acknowledged (s_waitcnt vmcnt(0) before each wave counts itself done),
// with no dirty line left in an XCD's L2 -- an agent-scope release per block per batch (an L2
// write-back, buffer_wbl2) took ~1.2 ms per batch for 512 blocks in the first build.  (16-B sc1
// stores stream at the plain rate, MI355X_MICROARCH.md.)
#ifndef FB_QUEUE_ST_AUX
#define FB_QUEUE_ST_AUX 16
#endif
constexpr int kQSt = FB_QUEUE_ST_AUX;  // cache-policy bits: sc1
// A batch's segments are handed to blocks in chunks from the slot's device counter (Q.head), each
// block holding its current chunk and the next: with a static share per block (k_parse_seg's rows)
// the blocks drifted apart by up to the ring's depth -- a batch took 362 us from its first block's
// start to its last block's end at depth 8 (tools/experiments/queue_trace.py) -- and the blocks
// ahead drained and waited while the ones behind ran on half a CU.
#ifndef FB_QUEUE_CHUNK
#define FB_QUEUE_CHUNK 16
#endif
constexpr uint32_t kQChunk = FB_QUEUE_CHUNK;  // segments per chunk
constexpr uint32_t kQRing = 8u;               // chunk ids per slot in the block's LDS (tagged)
// The chunk counters of a slot (kQHeads, each on its own 64-B line): with more than one, a block
// takes its XCD's chunks (c = j * kQHeads + x) and, once they are gone, the other XCDs'.  One counter
// carries 1,024 returning atomics per 24-us batch, about half a word's rate (MI355X_MICROARCH.md:
// ~88 per us), yet eight measured no faster (41.5 vs 41.8 Gpps over 512 batches) and the stealing at
// each batch's end lengthened its completion (profiles/r05_queue_ab.txt); chunks of 8 segments (2,048
// atomics per batch) cost 22 %, of 32 (coarser balance) 7 %.
#ifndef FB_QUEUE_HEADS
#define FB_QUEUE_HEADS 1
#endif
constexpr uint32_t kQHeads = FB_QUEUE_HEADS;
static_assert(kQHeads >= 1u && kQHeads <= 8u && (kQHeads & (kQHeads - 1u)) == 0u, "1, 2, 4 or 8 chunk counters");
static_assert(kQueueHeadWords >= kQHeads * 16u, "fb_internal.h: kQueueHeadWords");

struct QDesc {  // a ring slot's batch, cached in the block's LDS
    unsigned long long frames, offsets, out, seg, cls, stats;
    uint32_t frames_bytes, n, nseg, seq;  // seq: batch + 1 once the fields are valid
};
struct QLds {  // the block's queue state (per ring slot unless noted)
    QDesc desc[kQueueMax];
    uint32_t claim[kQueueMax];  // batch + 1 whose descriptor a wave has taken on to load
    uint32_t next[kQueueMax];   // the block's next position in the slot's batch (chunk i = L / kQChunk)
    unsigned long long chunk[kQueueMax * kQRing];  // (i + 1) << 32 | the batch's chunk number, or ~0u: none left
    uint32_t arr[kQueueMax];    // waves done with the slot's batch
    uint32_t acc[kQueueMax * 10u];
    uint32_t stop;              // the block leaves (host stop with nothing left, or idle)
    uint32_t tail;              // batches the block has seen published (one PCIe peek serves its waves)
};

__device__ __forceinline__ uint32_t u1st(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// The 100-MHz real-time counter, waited for in the same statement: s_memrealtime returns through
// lgkmcnt out of order with LDS operations, so a compiler-placed lgkmcnt(N) after the builtin form
// can read the register before it is written (the first queue build expired at once on garbage).
__device__ __forceinline__ unsigned long long rt_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long u1st64(unsigned long long x) {
    return (unsigned long long)u1st((uint32_t)x) | ((unsigned long long)u1st((uint32_t)(x >> 32)) << 32);
}
#ifdef FB_QUEUE_TRACE
#define QTRACE(stmt) do { stmt; } while (0)
__device__ __forceinline__ unsigned long long* qt(const QueueParams& Q, uint32_t what, uint64_t k) {
    return Q.trace + what * kQTraceN + (k % kQTraceN);
}
#else
#define QTRACE(stmt) do { } while (0)
#endif

// A chunk of the slot's batch for this block (~0u: none left): its XCD's counter, then the others'.
__device__ __forceinline__ uint32_t q_grab(const QueueParams& Q, uint32_t slot, uint32_t nch) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t x = kQHeads > 1u ? u1st(__builtin_amdgcn_s_getreg((31 << 11) | 20)) & (kQHeads - 1u) : 0u;  // XCC_ID
    for (uint32_t h = 0u; h < kQHeads; ++h) {
        const uint32_t y = (x + h) & (kQHeads - 1u);
        uint32_t r = 0u;
        if (lane == 0u)
            r = __hip_atomic_fetch_add(Q.head + slot * kQueueHeadWords + y * 16u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t c = u1st(r) * kQHeads + y;
        if (c < nch) return c;
    }
    return 0xFFFFFFFFu;
}

// One block at a time (whichever takes the poller word) reads the host's tail over PCIe and copies
// the new descriptors into the device ring -- 512 blocks polling the host each had every host access
// wait ~1 ms.  Returns the device ring's tail as this wave last saw it.  The host stores its tail before
// its stop word, so a stop followed (behind an acquire) by a tail with nothing new is final.
__device__ __forceinline__ unsigned long long q_refill(const QueueParams& Q, uint32_t k) {
    const uint32_t lane = threadIdx.x & 63u, R = Q.depth;
    // Every load here is relaxed and the poller word is released relaxed: these run on every poll, and on
    // gfx950 an agent release writes back (a system acquire invalidates) the XCD's L2 under the table
    // update kernels running beside a shared queue (bench single_batch_queue_table: 2.1 ms per 1M-frame
    // batch with acquire / release polls).  The tail and descriptor words are atomics (they bypass the
    // non-coherent caches); ordering is paid once per publication: a system acquire before the host's
    // descriptors are read, the device tail's release after they are copied.
    unsigned long long dt = __hip_atomic_load(&Q.d->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t got = 0u;
    if (lane == 0u) got = atomicCAS(&Q.d->poller, 0u, blockIdx.x + 1u) == 0u ? 1u : 0u;
    if (!u1st(got)) return dt;
    dt = __hip_atomic_load(&Q.d->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hs =
        u1st64(lane == 0u ? __hip_atomic_load(&Q.h->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull);
    const unsigned long long tl =
        u1st64(lane == 0u ? __hip_atomic_load(&Q.h->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull);
    QTRACE(if (lane == 0u) atomicAdd(qt(Q, kQtPolls, k), 1ull));
    if (tl > dt) {  // descriptors dt .. tl-1 (at most R: the host waits for slot reuse)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope: the host's descriptor stores)
        const uint32_t words = (uint32_t)min(tl - dt, (unsigned long long)R) * 8u;
        for (uint32_t w = lane; w < words; w += 64u) {
            const unsigned long long j = dt + w / 8u;
            const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&Q.h->desc[j & (R - 1u)]) + (w & 7u);
            unsigned long long* dst = reinterpret_cast<unsigned long long*>(&Q.d->desc[j & (R - 1u)]) + (w & 7u);
            *dst = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (lane == 0u) __hip_atomic_store(&Q.d->tail, tl, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        QTRACE(const unsigned long long now_ = rt_now();
               for (unsigned long long j = dt + lane; j < tl; j += 64u) *qt(Q, kQtPub, j) = now_);
        dt = tl;
    } else if (hs != 0ull) {
        // the two relaxed loads above may have been performed in either order: a stop is final only if
        // the tail read after it (behind an acquire, so after the stop) still has nothing new -- the
        // host stores its last tail before the stop (shutdown only: the fence's cost is paid once)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const unsigned long long tl2 =
            u1st64(lane == 0u ? __hip_atomic_load(&Q.h->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull);
        if (lane == 0u && tl2 <= dt) __hip_atomic_store(&Q.d->stop, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0u) __hip_atomic_store(&Q.d->poller, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return dt;
}

// Batch k's descriptor into the block's LDS, with the block's first chunk of it (false: the queue
// stops -- no batch k will come).
__device__ __forceinline__ bool q_ensure(const QueueParams& Q, QLds* L, uint32_t k) {
    const uint32_t lane = threadIdx.x & 63u, R = Q.depth, slot = k & (R - 1u);
    for (;;) {
        if (__hip_atomic_load(&L->desc[slot].seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == k + 1u) return true;
        if (__hip_atomic_load(&L->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        uint32_t won = 0u;
        if (lane == 0u) {
            const uint32_t expect = k >= R ? k - R + 1u : 0u;  // the slot's previous batch, or none
            won = atomicCAS(&L->claim[slot], expect, k + 1u) == expect ? 1u : 0u;
        }
        if (!u1st(won)) {  // another wave of the block loads it
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        // wait until batch k's descriptor is in the device ring
        const unsigned long long t0 = rt_now();
        unsigned long long dt;
        for (uint32_t spins = 0u;; ++spins) {
            // Idle polling is paced: every poll is a memory-side access to one line (the device tail,
            // the poller word), and a block's polls at s_sleep(2) -- 256 blocks of a shared queue, between
            // batches -- queue on that line's channel under the table update kernels beside the queue.
            // Past 64 polls (~0.1 ms with nothing published: the host is the slower side) only the first
            // 64 blocks keep polling every ~7 us; the others look every ~27 us and never take the poller
            // word (a batch's chunks are taken dynamically, so the early blocks start it alone).
            const bool slow = spins >= 64u && blockIdx.x >= 64u;
            if (slow) {
                for (int z = 0; z < 6; ++z) __builtin_amdgcn_s_sleep(127);
            }
            dt = __hip_atomic_load(&Q.d->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (relaxed poll)
            if (dt <= k && !slow && (spins < 8u || (spins & 3u) == 0u)) dt = q_refill(Q, k);
            if (dt > k) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // once, after the match
                if (lane == 0u) atomicMax(&L->tail, (uint32_t)dt);
                break;
            }
            const bool stop = __hip_atomic_load(&Q.d->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull;
            const unsigned long long now = rt_now();
            if (stop || now - t0 > Q.idle_ticks) {
                if (!stop && lane == 0u) {
                    // what the block saw when it left (pad words: diagnostics for the host)
                    __hip_atomic_store(&Q.h->pad[0], now - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&Q.h->pad[1], (unsigned long long)k | (unsigned long long)blockIdx.x << 32,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&Q.h->pad[2], dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&Q.h->status, kQueueExpired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (lane == 0u) __hip_atomic_store(&L->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return false;
            }
            if (spins < 8u) {
                __builtin_amdgcn_s_sleep(2);
            } else if (spins < 64u) {
                __builtin_amdgcn_s_sleep(32);
            } else {
                __builtin_amdgcn_s_sleep(127);  // (~6.8 us per poll once idle, a refill every 4th)
                __builtin_amdgcn_s_sleep(127);
            }
        }
        // lane j < 8 reads word j of the 64-B descriptor (fb_seg_batch) from the device ring
        const unsigned long long v =
            lane < 8u ? __hip_atomic_load(reinterpret_cast<const unsigned long long*>(&Q.d->desc[slot]) + lane,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : 0ull;
        QDesc& d = L->desc[slot];
        if (lane == 0u) d.frames = v;
        if (lane == 1u) d.frames_bytes = (uint32_t)v;
        if (lane == 2u) d.offsets = v;
        if (lane == 3u) {
            d.n = (uint32_t)v;
            d.nseg = ((uint32_t)v + 63u) / 64u;
        }
        if (lane == 4u) d.out = v;
        if (lane == 5u) d.seg = v;
        if (lane == 6u) d.cls = v;
        if (lane == 7u) d.stats = v;
        // the block's first chunk (its waves take the next ones, q_take)
        const uint32_t nseg0 = ((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 3) + 63u) / 64u;
        const uint32_t c0 = q_grab(Q, slot, (nseg0 + kQChunk - 1u) / kQChunk);
        if (lane == 0u) L->chunk[slot * kQRing] = (1ull << 32) | c0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0u) __hip_atomic_store(&d.seq, k + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        QTRACE(if (lane == 0u) atomicMin(qt(Q, kQtFirst, k), rt_now()));
        // the batch's first block keeps the device ring ahead of the waves: the descriptors the host
        // has published since are copied in now, before any wave runs out of batches
        if (c0 == 0u && dt < (unsigned long long)k + R) q_refill(Q, k);
        return true;
    }
}

// The block's next segment of the slot's batch (false: the batch has none left for this block).
// Position L of the block is offset L % kQChunk of the block's chunk L / kQChunk; the wave that
// takes a chunk's first position fetches the block's next chunk from the slot's device counter (after
// its own chunk is known, so the chunks of a block increase), or marks it empty once its own is.
// (Publishing the fetched chunk only at the wave's next position fetch, so the returned atomic's
// round trip overlaps a segment instead of draining the wave: 41.47 / 41.56 vs 41.45 / 41.43 Gpps
// over 512 batches, interleaved -- no gain, not kept; tools/experiments/queue_deferred_fetch.diff.)
__device__ __forceinline__ bool q_take(const QueueParams& Q, QLds* L, uint32_t slot, uint32_t* sg) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t v = 0u;
    if (lane == 0u) v = __hip_atomic_fetch_add(&L->next[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t pos = u1st(v), i = pos / kQChunk, o = pos % kQChunk;
    unsigned long long* ring = L->chunk + slot * kQRing;
    uint32_t c;
    for (;;) {
        const unsigned long long w = __hip_atomic_load(ring + i % kQRing, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((uint32_t)u1st64(w >> 32) == i + 1u) {
            c = u1st((uint32_t)w);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    const uint32_t nseg = u1st(L->desc[slot].nseg), nch = (nseg + kQChunk - 1u) / kQChunk;
    if (o == 0u) {
        uint32_t cn = 0xFFFFFFFFu;
        if (c < nch) cn = q_grab(Q, slot, nch);
        if (lane == 0u) __hip_atomic_store(ring + (i + 1u) % kQRing, ((unsigned long long)(i + 2u) << 32) | cn,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (c >= nch) return false;
    *sg = c * kQChunk + o;
    return *sg < nseg;
}

// This wave is done with batches [*arr_next, upto) -- its stores of them are complete (the caller
// waited) and its counters are in the block's LDS.  The block's last wave for a batch publishes the
// block's counters, resets the slot, writes the XCD's L2 back and counts the block; the batch's last
// block stores the completion word.
__device__ __forceinline__ void q_arrive(const QueueParams& Q, QLds* L, uint32_t* arr_next, uint32_t upto) {
    const uint32_t lane = threadIdx.x & 63u, R = Q.depth, G = gridDim.x;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the counters' LDS adds first)
    for (uint32_t j = *arr_next; j < upto; ++j) {
        const uint32_t slot = j & (R - 1u);
        uint32_t old = 0u;
        if (lane == 0u) old = __hip_atomic_fetch_add(&L->arr[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (u1st(old) != (uint32_t)kSegWaves - 1u) continue;
        if (lane < 5u) {  // the block's counters into the batch's five packed stats words (k_parse_seg's format)
            const unsigned long long lo = L->acc[slot * 10u + 2u * lane], hi = L->acc[slot * 10u + 2u * lane + 1u];
            unsigned long long* word = Q.tick + slot * 8u + lane;
            const unsigned long long add = (1ull << 54) | (hi << 27) | lo;
            const unsigned long long o = __hip_atomic_fetch_add(word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((o >> 54) == (unsigned long long)G - 1u) {  // this block completed the word: its fields
                const unsigned long long tot = o + add, m27 = (1ull << 27) - 1ull;
                const unsigned long long f_lo = tot & m27, f_hi = (tot >> 27) & m27;
                __hip_atomic_store(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fb_batch_stats* S = reinterpret_cast<fb_batch_stats*>(L->desc[slot].stats);
                // (system-scope stores: written through, like the records)
                auto put = [](uint64_t* p, unsigned long long v) {
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                };
                if (lane == 0u) {
                    put(&S->n_session, f_lo);
                    put(&S->n_filtered, f_hi);
                    put(&S->new_sessions, 0ull);
                    put(&S->updated_sessions, 0ull);
                    put(&S->error, __hip_atomic_load(Q.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    put(&S->reserved[0], 0ull);
                    put(&S->reserved[1], 0ull);
                    put(&S->reserved[2], 0ull);
                } else if (lane == 1u) {
                    put(&S->n_dns, f_lo);
                    put(&S->bad_offsets, f_hi);
                } else if (lane == 2u) {
                    put(&S->tcp_processed, f_lo);
                    put(&S->udp_processed, f_hi);
                } else if (lane == 3u) {
                    put(&S->ipv4_processed, f_lo);
                    put(&S->ipv6_processed, f_hi);
                } else {
                    put(&S->total_processed, f_lo);
                    put(&S->n_drop, f_hi);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // acknowledged before the block is counted
            }
        }
        if (lane < 10u) L->acc[slot * 10u + lane] = 0u;  // the slot's next batch starts from zero
        if (lane < kQRing) L->chunk[slot * kQRing + lane] = 0ull;
        if (lane == 0u) {
            L->next[slot] = 0u;
            L->arr[slot] = 0u;
        }
        // every wave of the block has its (write-through) stores of batch j acknowledged: count the block
        uint32_t ob = 0u;
        if (lane == 0u) ob = __hip_atomic_fetch_add(Q.blk_done + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        QTRACE(if (lane == 0u) {
            const unsigned long long now_ = rt_now();
            atomicMin(qt(Q, kQtArr0, j), now_);
            unsigned long long* b_ = Q.trace + kQTraceWords * kQTraceN + 4u * blockIdx.x;
            if (j == kQtB0 || j == kQtB1) b_[j == kQtB1] = now_;
            if (j == kQtB0) {
                b_[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
                b_[3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
            }
        });
        if (u1st(ob) == G - 1u) {  // the batch's last block (resets the slot's counters first)
            if (lane < kQHeads)
                __hip_atomic_store(Q.head + slot * kQueueHeadWords + lane * 16u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            QTRACE(if (lane == 0u) *qt(Q, kQtDone, j) = rt_now());
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (lane == 0u) {
                __hip_atomic_store(Q.blk_done + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&Q.h->cdone[slot], (unsigned long long)j + 1ull, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    *arr_next = upto > *arr_next ? upto : *arr_next;
}

// A wave's positions: (batch, segment) in increasing order -- batch gk, the wave's position count gt
// inside it (two static per wave, then the block's counter, as k_parse_seg hands them out).  block:
// wait for the batch to be published; otherwise a batch the host has not published ends it.
struct QPos {
    uint32_t k, sg, ok;
};
struct QGen {
    uint32_t gk, gt, known;
};
__device__ __forceinline__ QPos q_gen_slow(const QueueParams& Q, QLds* L, QGen* g, bool block, uint32_t* arr_next) {
    const uint32_t lane = threadIdx.x & 63u, R = Q.depth;
    for (;;) {
        if (g->gk >= g->known) {
            g->known = u1st(__hip_atomic_load(&L->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (g->gk >= g->known) {  // a peek at the device ring's tail (the poller keeps it current)
                uint32_t t = 0u;
                if (lane == 0u) {
                    t = (uint32_t)__hip_atomic_load(&Q.d->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // a peek
                    atomicMax(&L->tail, t);
                }
                g->known = u1st(t);
                if (g->gk >= g->known) {
                    if (!block) return QPos{g->gk, 0u, 0u};
                    QTRACE(if (lane == 0u) atomicAdd(qt(Q, kQtDrain, g->gk), 1ull));
                    // about to wait for a batch the host has not published: this wave (pipeline empty,
                    // counters flushed, stores complete -- the caller's drain) is done with every batch
                    // before it, including those it passed without a segment here; the host may be
                    // waiting for them before it publishes more
                    q_arrive(Q, L, arr_next, g->gk);
                }
            }
        }
        if (!q_ensure(Q, L, g->gk)) return QPos{g->gk, 0u, 0u};
        if (g->known <= g->gk) g->known = g->gk + 1u;
        g->gt = 1u;  // (inside batch gk: the main loop's fast path takes its positions)
        uint32_t sg;
        if (q_take(Q, L, g->gk & (R - 1u), &sg)) return QPos{g->gk, sg, 1u};
        ++g->gk;
        g->gt = 0u;
    }
}

__global__ __launch_bounds__(kSegThreads, kQueueWavesPerSimd) void k_parse_seg_queue(const QueueParams Q) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = u1st(tid >> 6), R = Q.depth;
    __shared__ uint4 s_cfg4[sizeof(DevConfig) / 16];
    __shared__ __attribute__((aligned(16))) unsigned long long s_stage[kSegWaves][64u * 7u];
    __shared__ QLds L;
    const DevConfig* cfg = reinterpret_cast<const DevConfig*>(s_cfg4);
    unsigned long long* stage = s_stage[wave];
    const unsigned long long lmask = (1ull << lane) - 1ull;
    constexpr uint32_t kOob = 0x80000000u;
    for (uint32_t k = tid; k < kQueueMax; k += kSegThreads) {
        L.desc[k].seq = 0u;
        L.claim[k] = 0u;
        L.next[k] = 0u;
        L.arr[k] = 0u;
    }
    for (uint32_t k = tid; k < kQueueMax * kQRing; k += kSegThreads) L.chunk[k] = 0ull;
    for (uint32_t k = tid; k < kQueueMax * 10u; k += kSegThreads) L.acc[k] = 0u;
    if (tid == 0u) {
        L.stop = 0u;
        L.tail = 0u;
        // count the block in; the last one tells the host that every block runs (host pad word 3)
        if (atomicAdd(&Q.d->pad[0], 1u) == gridDim.x - 1u)
            __hip_atomic_store(&Q.h->pad[3], (unsigned long long)gridDim.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(Q.cfg);
        constexpr uint32_t kCfg16 = kCfgLdsBytes / 16;
        for (uint32_t k = tid; k < kCfg16; k += kSegThreads) s_cfg4[k] = src[k];
        constexpr uint32_t kLanOff = offsetof(DevConfig, lan_v6) / 16, kOwnOff = offsetof(DevConfig, own) / 16;
        const uint32_t nl = Q.cfg->n_lan_v6 * (sizeof(LanV6) / 16), no = Q.cfg->n_own * (sizeof(fb_ip) / 16);
        for (uint32_t k = tid; k < nl; k += kSegThreads) s_cfg4[kLanOff + k] = src[kLanOff + k];
        for (uint32_t k = tid; k < no; k += kSegThreads) s_cfg4[kOwnOff + k] = src[kOwnOff + k];
    }
    __syncthreads();

    QGen g{0u, 0u, 0u};
    auto frames_rsrc = [&](uint32_t k) {
        const QDesc& d = L.desc[k & (R - 1u)];
        return __builtin_amdgcn_make_buffer_rsrc((void*)u1st64(d.frames), (short)0, (int)u1st(d.frames_bytes), 0x00020000);
    };
    auto load_q = [&](const QPos& p, uint2& q) {  // frame offsets of p's segment (invalid p: offsets[0])
        const QDesc& d = L.desc[p.k & (R - 1u)];
        const uint32_t* off = reinterpret_cast<const uint32_t*>(u1st64(d.offsets));
        const uint32_t n = u1st(d.n);
        const uint32_t i = p.ok ? p.sg * 64u + lane : 0u;
        q = make_uint2(off[min(i, n)], off[min(i + 1u, n)]);
    };
    auto vmov = [](uint32_t x) {
        uint32_t y;
        asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
        return y;
    };
    // counters of batch a_k (wave-uniform)
    uint32_t a_s = 0u, a_d = 0u, a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u, a_n = 0u, a_k = 0u, arr_next = 0u;
    auto flush = [&]() {
        const uint32_t a_tot = a_s + a_f;
        const uint32_t mine[10] = {a_s, a_f, a_d, a_b, a_t, a_tot - a_t, a_4, a_tot - a_4, a_tot, a_n - a_tot - a_d};
        if (lane < 10u) {
            uint32_t v = 0u;
#pragma unroll
            for (int k = 0; k < 10; ++k) v = lane == (uint32_t)k ? mine[k] : v;
            if (v) __hip_atomic_fetch_add(&L.acc[(a_k & (R - 1u)) * 10u + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        a_s = a_d = a_f = a_t = a_4 = a_b = a_n = 0u;
    };

    Hdr h;
    uint2 c = make_uint2(0u, 0u), q = make_uint2(0u, 0u);
    QPos cur{0u, 0u, 0u}, nxt{0u, 0u, 0u};
    for (;;) {
        if (!cur.ok) {
            // pipeline empty: everything this wave generated is processed; it is done with every batch
            // before g.gk; then wait for work (the only place a wave blocks)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            flush();
            q_arrive(Q, &L, &arr_next, g.gk);
            cur = q_gen_slow(Q, &L, &g, true, &arr_next);
            if (!cur.ok) break;
            nxt = q_gen_slow(Q, &L, &g, false, &arr_next);
            load_q(cur, q);
            load_headers1(frames_rsrc(cur.k), q.x, h);
            c = make_uint2(vmov(q.x), vmov(q.y));
            load_q(nxt.ok ? nxt : cur, q);
        }
        // the position after next: the fast path is a static position or a grab inside a known batch
        QPos aft{nxt.k, 0u, 0u};
        if (nxt.ok) {
            bool fast = false;
            if (g.gt) {  // a position inside the batch this wave is in
                uint32_t sg;
                if (q_take(Q, &L, g.gk & (R - 1u), &sg)) {
                    aft = QPos{g.gk, sg, 1u};
                    fast = true;
                } else {
                    ++g.gk;
                    g.gt = 0u;
                }
            }
            if (!fast) aft = q_gen_slow(Q, &L, &g, false, &arr_next);
        }
        if (cur.k != a_k) {  // the first segment of a later batch: the earlier ones are done here
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            flush();
            a_k = cur.k;
            q_arrive(Q, &L, &arr_next, cur.k);
        }
        const QDesc& D = L.desc[cur.k & (R - 1u)];
        const uint32_t n = u1st(D.n), fbytes = u1st(D.frames_bytes);
        const uint32_t ls = cur.sg, i = ls * 64u + lane;
        const bool valid = i < n;
        Pkt kk;
        process_frame(frames_rsrc(cur.k), cfg, cfg, h, valid ? c.x : 1u, valid ? c.y : 0u, fbytes, i, kk);
        const bool is_s = valid && kk.cls == FB_CLASS_SESSION;
        const bool is_d = valid && kk.cls == FB_CLASS_DNS;
        const bool is_f = valid && kk.cls == FB_CLASS_FILTERED;
        const bool counted = is_s || is_f;
        const unsigned long long m_sess = __ballot(is_s), m_dns = __ballot(is_d);
        const uint32_t cs = (uint32_t)__popcll(m_sess), cd = (uint32_t)__popcll(m_dns);
        if (is_s) {
            unsigned long long* dd = stage + (size_t)__popcll(m_sess & lmask) * 7;
#pragma unroll
            for (int w = 0; w < 7; ++w) dd[w] = (unsigned long long)kk.w[2 * w] | ((unsigned long long)kk.w[2 * w + 1] << 32);
        }
        __builtin_amdgcn_wave_barrier();
        // prefetch: the next segment's headers (offsets already here), the offsets of the one after
        // (an invalid position reads its batch's offsets[0] / the frame at 0: harmless, never used)
        load_headers1(frames_rsrc(nxt.ok ? nxt.k : cur.k), nxt.ok ? q.x : 0u, h);
        c = make_uint2(vmov(q.x), vmov(q.y));
        load_q(aft.ok ? aft : cur, q);
        {   // stores (as k_parse_seg): 4 x 16 B of records, the 8-B tail, one DNS record, the count, the class
            uint8_t* out = reinterpret_cast<uint8_t*>(u1st64(D.out)) + (size_t)ls * kSegBytes;
            const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)kSegBytes, 0x00020000);
            uint32_t* segw = reinterpret_cast<uint32_t*>(u1st64(D.seg));
            uint8_t* clsp = reinterpret_cast<uint8_t*>(u1st64(D.cls));
            const __amdgpu_buffer_rsrc_t r_seg =
                __builtin_amdgcn_make_buffer_rsrc(segw, (short)0, (int)(((n + 63u) / 64u) * 4u), 0x00020000);
            const __amdgpu_buffer_rsrc_t r_cls = __builtin_amdgcn_make_buffer_rsrc(clsp, (short)0, clsp ? (int)n : 0, 0x00020000);
            const uint32_t words = cs * 7u, body = words >> 1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t cc = lane + 64u * j;
                const uint32_t src = min(cc, 223u);
                const unsigned long long x = stage[2u * src], y = stage[2u * src + 1u];
                const u32x4 v = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(v, r_out, cc < body ? cc * 16u : kOob, 0, kQSt);
            }
            {
                const bool tail = (words & 1u) && lane == 0u;
                const unsigned long long x = stage[words ? words - 1u : 0u];
                const u32x2 v = {(uint32_t)x, (uint32_t)(x >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(v, r_out, tail ? (words - 1u) * 8u : kOob, 0, kQSt);
            }
            {
                const u32x4 v = {kk.w[0], kk.w[1], kk.w[2], kk.w[3]};
                __builtin_amdgcn_raw_buffer_store_b128(
                    v, r_out, is_d ? kSegBytes - 16u * (1u + (uint32_t)__popcll(m_dns & lmask)) : kOob, 0, kQSt);
            }
            __builtin_amdgcn_raw_buffer_store_b32(cs | (cd << 16), r_seg, lane == 0u ? ls * 4u : kOob, 0, kQSt);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)kk.cls, r_cls, valid ? i : kOob, 0, kQSt);
        }
        __builtin_amdgcn_wave_barrier();  // stage reads of this segment before the next writes
        a_s += cs;
        a_d += cd;
        a_f += __popcll(__ballot(is_f));
        a_t += __popcll(__ballot(counted && kk.tcp));
        a_4 += __popcll(__ballot(counted && kk.v4));
        a_b += __popcll(__ballot(valid && kk.bad));
        a_n += __popcll(__ballot(valid));
        cur = nxt;
        nxt = aft;
    }
}

hipError_t occupancy_parse_seg_queue(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_parse_seg_queue, kSegThreads, 0);
}
hipError_t launch_parse_seg_queue(const QueueParams& q, uint32_t grid, hipStream_t s) {
    if (q.depth == 0u || q.depth > kQueueMax) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_parse_seg_queue, dim3(grid), dim3(kSegThreads), 0, s, q);
    return hipGetLastError();
}

}  // namespace fbk
