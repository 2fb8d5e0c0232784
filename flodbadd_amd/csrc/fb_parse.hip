// fb_parse.hip -- gfx950 parse + classify kernels: k_parse_seg (streaming, per-wavefront
// compaction into 64-frame output segments) and k_parse_ws (role-specialised pipeline with one
// batch-wide compaction).
//
// One wavefront lane per frame.  Replaces, per frame:
//   parse_packet_pcap                 src/packets.rs:603-802 (pnet_packet 0.35.0 decode)
//   service-port direction + key      src/packets.rs:232-311 (get_name_from_port, port_vulns.rs:213)
//   is_originator                     src/packets.rs:316-319
//   Local/Global session filter       src/packets.rs:321-327, sessions.rs:660-672, ip.rs:199-242
//   PACKET_STATS pre-filter counters  src/packets.rs:211-227
//   map_tcp_flags (history char)      src/packets.rs:561-601
//
// Both kernels share the device functions below (header decode, classification, history char)
// and differ only in how the emitted records are laid out.  Loads: four unaligned header loads
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

__device__ __forceinline__ fb_dns_out make_fb_dns(const Pkt& k) {
    fb_dns_out d;
    d.pkt_index = k.w[0];
    d.payload_offset = k.w[1];
    d.payload_length = k.w[2];
    d.protocol = (uint8_t)(k.w[3] & 0xffu);
    d.family = (uint8_t)(k.w[3] >> 8);
    d.reserved = 0;
    return d;
}

__device__ __forceinline__ unsigned long long ald(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned long long kCountMask = (1ull << 56) - 1ull;  // [dns:28 | session:28]
__device__ __forceinline__ uint32_t tag_of(unsigned long long w) { return (uint32_t)(w >> 56); }

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Ablation switches (tools/ubench_ws.hip); the product instantiates kFlagsProduct.
constexpr uint32_t kFlagsProduct = 0u;
constexpr uint32_t kNoLookback = 1u;  // base offsets = tile start (wrong output, timing only)
constexpr uint32_t kNoStore = 2u;     // no record / dns stores (timing only)
constexpr uint32_t kStamps = 4u;      // per-unit s_memrealtime stamps into P.dbg
constexpr uint32_t kPartOut = 8u;     // k_parse_seg: also the flow-table partition of each SESSION
                                      // record slot (P.rec_part), for the update that follows

constexpr unsigned long long kIncBit = 1ull << 55;
constexpr unsigned long long kCnt28 = (1ull << 28) - 1ull;
__device__ __forceinline__ unsigned long long st_counts(unsigned long long w) {
    return (w & kCnt28) | (((w >> 28) & ((1ull << 27) - 1ull)) << 28);
}
__device__ __forceinline__ unsigned long long st_pack(uint32_t ep, bool inc, unsigned long long c) {
    return ((unsigned long long)ep << 56) | (inc ? kIncBit : 0ull) | (c & kCnt28) |
           (((c >> 28) & ((1ull << 27) - 1ull)) << 28);
}

// Batch totals (the wave owning the last tile): `tot_c` = inclusive [dns|session] count
// through the last tile; the pre-filter counters come from every wave's epoch-tagged slot.
__device__ void write_batch_stats(const ParseParams& P, unsigned long long tot_c, uint32_t W) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t ep = P.epoch;
    unsigned long long sf = 0ull, sb = 0ull;
    uint32_t spins = 0u;
    for (uint32_t q0 = 0; q0 < W; q0 += 64u) {
        const uint32_t q = q0 + lane;
        const bool own = q < W;
        unsigned long long a = own ? ald(P.wstat + 2 * q) : 0ull, b = own ? ald(P.wstat + 2 * q + 1) : 0ull;
        for (;;) {
            const bool ok = !own || (tag_of(a) == ep && tag_of(b) == ep);
            if (__ballot(!ok) == 0ull) break;
            if (++spins > (1u << 20)) { if (lane == 0u) atomicOr(P.error, 1u); break; }
            __builtin_amdgcn_s_sleep(8);
            if (!ok) { a = ald(P.wstat + 2 * q); b = ald(P.wstat + 2 * q + 1); }
        }
        sf += own ? (a & kCountMask) : 0ull;
        sb += own ? (b & kCountMask) : 0ull;
    }
    sf = wave_sum64(sf);
    sb = wave_sum64(sb);
    if (lane == 0u) {
        fb_batch_stats* S = P.stats;
        const unsigned long long ns = tot_c & ((1ull << 28) - 1ull), nd = tot_c >> 28;
        const unsigned long long nf = sf & ((1ull << 28) - 1ull), nt = sf >> 28;
        const unsigned long long n4 = sb & ((1ull << 28) - 1ull), nb = sb >> 28;
        const unsigned long long tot = ns + nf;
        S->total_processed = tot;
        S->tcp_processed = nt;
        S->udp_processed = tot - nt;
        S->ipv4_processed = n4;
        S->ipv6_processed = tot - n4;
        S->new_sessions = 0ull;
        S->updated_sessions = 0ull;
        S->n_session = ns;
        S->n_dns = nd;
        S->n_drop = (unsigned long long)P.n - tot - nd;
        S->n_filtered = nf;
        S->bad_offsets = nb;
        S->error = __hip_atomic_load(P.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S->reserved[0] = S->reserved[1] = S->reserved[2] = 0ull;
    }
}

__device__ __forceinline__ void load_headers1(__amdgpu_buffer_rsrc_t rs, uint32_t o, Hdr& h) {
#if FB_HDR_ALIGNED
    const uint32_t a = (o + 10u) & ~3u;
    h.A = ld16(rs, a);
    h.B = ld16(rs, a + 16u);
    h.C = ld16(rs, a + 32u);
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

// ---- round look-back (k_parse_ws) -----------------------------------------------------------
// Units are dealt round-robin: round r = units [r*G, (r+1)*G), unit r*G + b belongs to block b.
// The exclusive prefix of unit u = r*G + b is  sum(RSUM[0..r-1]) + sum(AGG[r*G .. u-1]):  one
// probe of b + r epoch-tagged words, with no chain of inclusive prefixes from round to round
// (each link of such a chain costs a memory round trip, ~2-3 us on a CU that streams, and the
// chain grows with the round count).  RSUM[r] is published by the look-back of the round's last
// unit (b = G-1), which reads every other AGG of the round anyway.  Not-ready words are
// re-polled by their lanes together with exponential back-off.
template <uint32_t FLAGS>
__device__ unsigned long long lookback_round(const ParseParams& P, uint32_t r, uint32_t b, uint32_t G,
                                             unsigned long long agg, uint32_t& spins) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t ep = P.epoch;
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc((void*)(P.tagg + (size_t)r * G), (short)0, (int)(b * 8u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)P.rsum, (short)0, (int)(r * 8u), 0x00020000);
    auto word = [&](uint32_t idx) {  // idx < b: AGG of round-mate idx; else RSUM[idx - b]
        const u32x2 x = idx < b ? __builtin_amdgcn_raw_buffer_load_b64(ra, idx * 8u, 0, 16)
                                : __builtin_amdgcn_raw_buffer_load_b64(rr, (idx - b) * 8u, 0, 16);
        return (unsigned long long)x.x | ((unsigned long long)x.y << 32);
    };
    const uint32_t m = b + r;
    unsigned long long sa = 0ull, sr = 0ull;  // AGG part, RSUM part
    spins = 0u;
    for (uint32_t c0 = 0; c0 < m; c0 += 256u) {
        unsigned long long v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t idx = c0 + 64u * q + lane;
            v[q] = idx < m ? word(idx) : ((unsigned long long)ep << 56);
        }
        for (;;) {
            bool ready = true;
#pragma unroll
            for (int q = 0; q < 4; ++q) ready &= tag_of(v[q]) == ep;
            if (__ballot(!ready) == 0ull) break;
            if (++spins > (1u << 16)) { if (lane == 0u) atomicOr(P.error, 1u); return 0ull; }
            for (uint32_t z = 0; z < min(spins, 4u); ++z) __builtin_amdgcn_s_sleep(4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t idx = c0 + 64u * q + lane;
                if (tag_of(v[q]) != ep) v[q] = word(idx);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t idx = c0 + 64u * q + lane;
            if (idx < b) sa += st_counts(v[q]);
            else sr += st_counts(v[q]);
        }
    }
    sa = wave_sum64(sa);
    sr = wave_sum64(sr);
    // the round's last unit: round r is complete, publish its sum (round-mates' AGGs + own)
    if (b == G - 1u && lane == 0u) ast(P.rsum + r, st_pack(ep, false, sa + agg));
    return sa + sr;
}

// ============================================================================================
// k_parse_ws -- role-specialised block pipeline (the product kernel).
//
// A block (one per CU) = kWsLoad loader waves + kWsLb look-back waves + kWsStore storer waves.
// A unit = kWsLoad x kWsU wave-tiles x 64 frames (loader wave w owns frames [w*64U, (w+1)*64U)
// of the unit, so packet order = (wave, tile, lane)); block b owns units b, b+G, b+2G, ...
// (k-th unit of the block = b + k*G, staged in LDS slot k % kWsSlots).  The roles run
// decoupled, each at its own pace, handing units over through monotonic LDS counters (no
// block barrier in the loop, so a slow look-back stalls nobody until the slots run out):
//   loader waves   : wait until slot k%S is free -> classify unit k (its headers were issued two
//                    units earlier) -> stage SESSION / DNS records, compacted per wave, + counts
//                    -> signal STAGED -> issue the offset loads of unit k+3 and the header loads
//                    of unit k+2
//   look-back wave : (unit k = j mod kWsLb for wave j) wait STAGED -> publish AGG, decoupled
//                    look-back, publish INC -> prefix to the slot -> signal READY
//   storer waves   : wait READY -> copy the slot's records to the output with coalesced 16-B
//                    stores -> signal FREE
// Loader waves issue only loads and storer waves only stores, so no wave's vmcnt wait covers
// the other role's traffic: two units of header loads stay in flight per loader wave.
// ============================================================================================
#ifndef FB_WS_LOAD
#define FB_WS_LOAD 8
#endif
#ifndef FB_WS_U
#define FB_WS_U 1
#endif
#ifndef FB_WS_STORE
#define FB_WS_STORE 4
#endif
#ifndef FB_WS_LB
#define FB_WS_LB 2
#endif
#ifndef FB_WS_SLOTS
#define FB_WS_SLOTS 5
#endif
#ifndef FB_WS_DEPTH
#define FB_WS_DEPTH 2
#endif
constexpr int kWsLoad = FB_WS_LOAD;
constexpr int kWsU = FB_WS_U;
constexpr int kWsStore = FB_WS_STORE;
constexpr int kWsLb = FB_WS_LB;
constexpr int kWsSlots = FB_WS_SLOTS;
constexpr int kWsDepth = FB_WS_DEPTH;  // units of header loads in flight per loader wave
constexpr int kWsThreads = 64 * (kWsLoad + 1 + kWsLb + kWsStore);  // + 1 AGG publisher wave
#ifndef FB_WS_LBWIN
#define FB_WS_LBWIN 8
#endif
constexpr int kWsLbWin = FB_WS_LBWIN;  // look-back probe window, x64 units
constexpr uint32_t kWsWF = 64u * kWsU;         // frames per loader wave per unit
constexpr uint32_t kWsUnit = kWsWF * kWsLoad;  // frames per unit

// Per loader wave, one 64U x 56-B region: SESSION records compacted from the front, DNS records
// (16 B) from the back -- a frame is one or the other, so they never overlap.
struct WsSlot {
    unsigned long long rec[kWsLoad][kWsWF * 7];
    uint32_t cnt[kWsLoad][4];  // sessions, dns, filtered|tcp<<16, v4|bad<<16
    unsigned long long agg;    // [dns:28 | session:28] of the unit
    unsigned long long excl;   // [dns:28 | session:28] prefix of the unit
};
struct WsSync {               // monotonic hand-off counters per slot
    uint32_t cfg;               // + 1 per copying wave once the configuration is in LDS
    uint32_t staged[kWsSlots];  // + 1 per loader wave per unit
    uint32_t agged[kWsSlots];   // = generation + 1 once the AGG is published and in the slot
    uint32_t ready[kWsSlots];   // = generation + 1 once the prefix is in the slot
    uint32_t freed[kWsSlots];   // + 1 per storer wave per unit
};
__device__ __forceinline__ uint4* ws_dns(WsSlot& S, uint32_t w, uint32_t j) {
    return reinterpret_cast<uint4*>(&S.rec[w][kWsWF * 7]) - 1 - j;
}
__device__ __forceinline__ const uint4* ws_dns(const WsSlot& S, uint32_t w, uint32_t j) {
    return reinterpret_cast<const uint4*>(&S.rec[w][kWsWF * 7]) - 1 - j;
}
// s_barrier that drains this wave's LDS traffic only (never vector memory).
__device__ __forceinline__ void ws_tick() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Signal after this wave's LDS writes / reads of a slot: drain LDS (not vector memory), then add.
__device__ __forceinline__ void lds_signal(uint32_t* p, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63u) == 0u) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t target) {
    while (lds_ld(p) < target) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// kStamps (ablation builds): P.dbg[(b * kWsDbgUnits + k) * 4 + role] = s_memrealtime at
// role 3: loader wave 0 starts unit k, 0: loader wave 0 staged it, 1: its INC published,
// 2: storer wave 0 done with it.
constexpr uint32_t kWsDbgUnits = 64;
template <bool PARSED, uint32_t FLAGS = kFlagsProduct>
__global__ __launch_bounds__(kWsThreads) void k_parse_ws(const ParseParams P) {
    constexpr int U = kWsU;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t G = gridDim.x, T = P.num_tiles, b = blockIdx.x;
    const uint32_t K = (T - b + G - 1u) / G;  // units of this block (grid <= T, so K >= 1)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;
    auto stamp = [&](uint32_t k, int role) {
        if constexpr ((FLAGS & kStamps) != 0u)
            if (lane == 0u && k < kWsDbgUnits - 1u) P.dbg[(b * kWsDbgUnits + k) * 4 + role] = __builtin_amdgcn_s_memrealtime();
    };
    // block-level stamps in the last debug unit: 3 entry, 0 loader exit, 1 look-back exit, 2 storer exit
    auto bstamp = [&](int role) {
        if constexpr ((FLAGS & kStamps) != 0u)
            if (lane == 0u) P.dbg[(b * kWsDbgUnits + kWsDbgUnits - 1u) * 4 + role] = __builtin_amdgcn_s_memrealtime();
    };
    if (tid == 0u) bstamp(3);

    __shared__ uint4 s_cfg4[sizeof(DevConfig) / 16];  // header + bitmap + the used table entries
    __shared__ WsSlot s_slot[kWsSlots];
    __shared__ WsSync s_sync;
    const DevConfig* cfg = reinterpret_cast<const DevConfig*>(s_cfg4);
    const DevConfig* gcfg = cfg;  // tables read from LDS too (a global read here would wait for
                                  // every in-flight header load)
    constexpr uint32_t kCopyWaves = (uint32_t)(kWsThreads / 64 - kWsLoad);
    if (tid < sizeof(WsSync) / 4) reinterpret_cast<uint32_t*>(&s_sync)[tid] = 0u;
    ws_tick();  // counters zeroed (LDS-only barrier; nothing is in flight yet)
    const bool is_loader = wave < (uint32_t)kWsLoad;
    const unsigned long long lmask = (1ull << lane) - 1ull;

    if (is_loader) {
        // ================================ loader waves ================================
        // kWsDepth units of header loads in flight per wave.  Register set d (headers h, the
        // unit's offsets c, and q = the offsets of the unit it fetches next) serves units
        // k = d mod D; the loop is unrolled by D, so no set is indexed at run time.  After
        // classifying unit k with set X:  X.h <- headers(k+D) from X.q (waited for with the
        // younger loads of D-1 other units in flight) ; X.c <- X.q (explicit v_mov: the
        // allocator cannot rename q across the loop, so no back-edge copy waits on a pending
        // load) ; X.q <- offsets(k+2D).  The prefetch is unconditional (past the last unit the
        // offsets clamp to offsets[n] and the header loads fall outside the buffer), so every
        // path issues the same VMEM sequence and the compiler's vmcnt bookkeeping stays exact.
        constexpr int D = kWsDepth;
        struct Set {
            Hdr h[U];
            uint2 c[U];
            uint2 q[U];
        };
        Set SS[D];
        uint4 pin[U][4];
        auto vmov = [](uint32_t x) {
            uint32_t y;
            asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
            return y;
        };
        auto frame0 = [&](uint32_t k) { return (b + k * G) * kWsUnit + wave * kWsWF; };
        auto load_offs = [&](uint32_t k, uint2 (&dst)[U]) {
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = frame0(k) + r * 64u + lane;
                dst[r] = make_uint2(P.offsets[min(i, P.n)], P.offsets[min(i + 1u, P.n)]);
            }
        };
        auto load_parsed = [&](uint32_t k) {
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = min(frame0(k) + r * 64u + lane, P.n - 1u);
                const uint4* qq = reinterpret_cast<const uint4*>(P.parsed + i);
                pin[r][0] = qq[0];
                pin[r][1] = qq[1];
                pin[r][2] = qq[2];
                const uint2 t = *reinterpret_cast<const uint2*>(qq + 3);
                pin[r][3] = make_uint4(t.x, t.y, 0u, 0u);
            }
        };
        auto fetch = [&](Set& X, uint32_t k_next_q) {  // headers from X.q, then X.q <- offs(k_next_q)
#pragma unroll
            for (int r = 0; r < U; ++r) {
                load_headers1(rs, X.q[r].x, X.h[r]);
                X.c[r] = make_uint2(vmov(X.q[r].x), vmov(X.q[r].y));
            }
            load_offs(k_next_q, X.q);
        };
        if constexpr (!PARSED) {
#pragma unroll
            for (int d = 0; d < D; ++d) load_offs((uint32_t)d, SS[d].q);
#pragma unroll
            for (int d = 0; d < D; ++d) fetch(SS[d], (uint32_t)(d + D));
        } else {
            load_parsed(0);
        }
        auto step = [&](uint32_t k, Set& X) {
            const uint32_t sl = k % kWsSlots, g = k / kWsSlots;
            stamp(k, 3);
            lds_wait_ge(&s_sync.cfg, kCopyWaves);           // configuration in LDS (first unit)
            lds_wait_ge(&s_sync.freed[sl], g * kWsStore);  // unit k - S fully copied out
            WsSlot& S = s_slot[sl];
            unsigned long long* stage = S.rec[wave];
            const uint32_t f0 = frame0(k);
            uint32_t cs = 0u, cd = 0u, wf = 0u, wt = 0u, w4 = 0u, wb = 0u;
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = f0 + r * 64u + lane;
                const bool valid = i < P.n;
                Pkt kk;
                if constexpr (!PARSED) {
                    process_frame(rs, cfg, gcfg, X.h[r], valid ? X.c[r].x : 1u, valid ? X.c[r].y : 0u,
                                  P.frames_bytes, i, kk);
                } else {
                    const uint4 a = pin[r][0], bb = pin[r][1], c = pin[r][2], d = pin[r][3];
                    const uint32_t src[4] = {a.x, a.y, a.z, a.w}, dst[4] = {bb.x, bb.y, bb.z, bb.w};
                    const uint32_t proto = c.y & 0xffu, fam = (c.y >> 8) & 0xffu;
                    kk.bad = false;
                    kk.cls = FB_CLASS_DROP;
                    kk.tcp = kk.v4 = false;
                    if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                        classify_session(cfg, gcfg, proto, fam, src, dst, c.x & 0xffffu, c.x >> 16, (d.x >> 8) & 1u,
                                         d.x & 0xffu, c.z, c.w, d.y, kk);
                }
                const bool is_s = valid && kk.cls == FB_CLASS_SESSION;
                const bool is_d = valid && kk.cls == FB_CLASS_DNS;
                const bool is_f = valid && kk.cls == FB_CLASS_FILTERED;
                const bool counted = is_s || is_f;
                const unsigned long long m_sess = __ballot(is_s), m_dns = __ballot(is_d);
                if (is_s) {
                    unsigned long long* dd = stage + (size_t)(cs + __popcll(m_sess & lmask)) * 7;
#pragma unroll
                    for (int w = 0; w < 7; ++w)
                        dd[w] = (unsigned long long)kk.w[2 * w] | ((unsigned long long)kk.w[2 * w + 1] << 32);
                }
                if (is_d) *ws_dns(S, wave, cd + __popcll(m_dns & lmask)) = make_uint4(kk.w[0], kk.w[1], kk.w[2], kk.w[3]);
                cs += (uint32_t)__popcll(m_sess);
                cd += (uint32_t)__popcll(m_dns);
                wf += __popcll(__ballot(is_f));
                wt += __popcll(__ballot(counted && kk.tcp));
                w4 += __popcll(__ballot(counted && kk.v4));
                wb += __popcll(__ballot(valid && kk.bad));
                if (valid && P.cls) P.cls[i] = (uint8_t)kk.cls;
            }
            if (lane == 0u) {
                S.cnt[wave][0] = cs;
                S.cnt[wave][1] = cd;
                S.cnt[wave][2] = wf | (wt << 16);
                S.cnt[wave][3] = w4 | (wb << 16);
            }
            lds_signal(&s_sync.staged[sl], 1u);
            stamp(k, 0);
            if constexpr (!PARSED) fetch(X, k + 2u * D);
            else load_parsed(k + 1u);
        };
        uint32_t k = 0;
        for (; k + D <= K; k += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) step(k + d, SS[d]);
        }
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if (k + d < K) step(k + d, SS[d]);
        if (wave == 0u) bstamp(0);
    } else {
        // non-loader waves copy the configuration header + service bitmap into LDS while the
        // loaders' first header loads are in flight
        const uint32_t t2 = tid - 64u * kWsLoad;
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        for (uint32_t q = t2; q < kCfgLdsBytes / 16; q += 64u * kCopyWaves) s_cfg4[q] = src[q];
        // table entries in use only (sizes are uniform: scalar loads of the header)
        constexpr uint32_t kLanOff = offsetof(DevConfig, lan_v6) / 16, kOwnOff = offsetof(DevConfig, own) / 16;
        const uint32_t nl = P.cfg->n_lan_v6 * (sizeof(LanV6) / 16), no = P.cfg->n_own * (sizeof(fb_ip) / 16);
        for (uint32_t q = t2; q < nl; q += 64u * kCopyWaves) s_cfg4[kLanOff + q] = src[kLanOff + q];
        for (uint32_t q = t2; q < no; q += 64u * kCopyWaves) s_cfg4[kOwnOff + q] = src[kOwnOff + q];
        if (b == 0u && t2 == 0u) *P.error_next = 0u;  // other parity's word, for the next launch
        lds_signal(&s_sync.cfg, 1u);
    }
    if (is_loader) {
    } else if (wave == (uint32_t)kWsLoad) {
        // ============================== AGG publisher wave ==============================
        // Publishes every unit's aggregate as soon as it is staged (a look-back of another
        // block may be waiting for it), and sums the block's pre-filter counters.
        uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t sl = k % kWsSlots, g = k / kWsSlots;
            WsSlot& S = s_slot[sl];
            lds_wait_ge(&s_sync.staged[sl], (g + 1u) * kWsLoad);
            uint32_t bs = 0u, bd = 0u;
#pragma unroll
            for (int w = 0; w < kWsLoad; ++w) {
                bs += S.cnt[w][0];
                bd += S.cnt[w][1];
                a_f += S.cnt[w][2] & 0xFFFFu;
                a_t += S.cnt[w][2] >> 16;
                a_4 += S.cnt[w][3] & 0xFFFFu;
                a_b += S.cnt[w][3] >> 16;
            }
            const unsigned long long agg = (unsigned long long)bs | ((unsigned long long)bd << 28);
            if (lane == 0u) {
                if (!(FLAGS & kNoLookback)) ast(P.tagg + b + k * G, st_pack(ep, false, agg));
                S.agg = agg;
                __hip_atomic_store(&s_sync.agged[sl], g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (lane == 0u && !(FLAGS & kNoLookback)) {
            ast(P.wstat + 2 * b, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
            ast(P.wstat + 2 * b + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
        }
    } else if (wave < (uint32_t)(kWsLoad + 1 + kWsLb)) {
        // ================================ look-back waves ================================
        const uint32_t j = wave - (uint32_t)kWsLoad - 1u;
        unsigned long long tot_c = 0ull;
        for (uint32_t k = j; k < K; k += kWsLb) {
            const uint32_t sl = k % kWsSlots, g = k / kWsSlots;
            WsSlot& S = s_slot[sl];
            const uint32_t u = b + k * G;
            lds_wait_ge(&s_sync.agged[sl], g + 1u);
            const unsigned long long agg = S.agg;
            unsigned long long excl;
            if constexpr ((FLAGS & kNoLookback) != 0u) {
                excl = (unsigned long long)u * kWsUnit;
            } else {
                uint32_t spins;
                excl = lookback_round<kFlagsProduct>(P, k, b, G, agg, spins);
            }
            if (lane == 0u) {
                S.excl = excl;
                __hip_atomic_store(&s_sync.ready[sl], g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            stamp(k, 1);
            if (u == T - 1u) tot_c = excl + agg;  // the batch's last unit: inclusive totals
        }
        // the wave that owns the batch's last unit sums every block's pre-filter counters
        if ((T - 1u) % G == b && (K - 1u) % kWsLb == j && P.stats && !(FLAGS & kNoLookback))
            write_batch_stats(P, tot_c, G);
        if (j == 0u) bstamp(1);
    } else {
        // ================================ storer waves ================================
        // Storer wave v copies loader regions v, v+SW, ...: region w's records go to output
        // records [base + ps[w], +cs_w) with 16-B stores (8-B head/tail where the 56-B record
        // boundary is not 16-B aligned); its DNS records likewise, 16 B each.
        const uint32_t sw = wave - (uint32_t)(kWsLoad + 1 + kWsLb);
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t sl = k % kWsSlots, g = k / kWsSlots;
            lds_wait_ge(&s_sync.ready[sl], g + 1u);
            const WsSlot& S = s_slot[sl];
            if (!(FLAGS & kNoStore)) {
                const unsigned long long ex = S.excl;
                uint32_t base_s = (uint32_t)(ex & kCnt28), base_d = (uint32_t)(ex >> 28);
                for (uint32_t w = 0; w < (uint32_t)kWsLoad; ++w) {
                    const uint32_t cs = S.cnt[w][0], cd = S.cnt[w][1];
                    if ((w % kWsStore) == sw) {
                        const unsigned long long* src = S.rec[w];
                        if (P.out && cs) {
                            unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7u;
                            const uint32_t words = cs * 7u, head = base_s & 1u, body = (words - head) >> 1;
                            if (head && lane == 0u) g8[0] = src[0];
                            uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                            for (uint32_t c = lane; c < body; c += 64u) {
                                const unsigned long long x = src[head + 2u * c], y = src[head + 2u * c + 1u];
                                g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                            }
                            if (lane == 0u && head + 2u * body < words) g8[words - 1u] = src[words - 1u];
                        }
                        if (P.dns) {
                            for (uint32_t jd = lane; jd < cd; jd += 64u) {
                                const uint4 v = *ws_dns(S, w, jd);
                                fb_dns_out d;
                                d.pkt_index = v.x;
                                d.payload_offset = v.y;
                                d.payload_length = v.z;
                                d.protocol = (uint8_t)(v.w & 0xffu);
                                d.family = (uint8_t)(v.w >> 8);
                                d.reserved = 0;
                                P.dns[base_d + jd] = d;
                            }
                        }
                    }
                    base_s += cs;
                    base_d += cd;
                }
            }
            lds_signal(&s_sync.freed[sl], 1u);
            if (sw == 0u) stamp(k, 2);
        }
        if (sw == 0u) bstamp(2);
    }
}

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

// Ablations (tools/ubench_ws.hip): kNoStore drops every store, kNoLookback here means "no
// classification" (each frame becomes a SESSION record of raw header words).
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
    __shared__ unsigned long long s_stage[kSegWaves][64 * 7];
    __shared__ uint32_t s_acc[kAcc + 1];  // per batch: block counters (see the stats section); wave arrivals
    const DevConfig* cfg = reinterpret_cast<const DevConfig*>(s_cfg4);
    const unsigned long long lmask = (1ull << lane) - 1ull;
    unsigned long long* stage = s_stage[wave];
    // kStamps: P.dbg[(b * kSegWaves + wave) * 16 + slot]: 0 entry, 1 prologue done, 2.. end of
    // iteration j (j < 12), 14 stats start, 15 exit
    auto sstamp = [&](uint32_t slot) {
        if constexpr ((FLAGS & kStamps) != 0u)
            if (lane == 0u && slot < 16u)
                P.dbg[((size_t)b * kSegWaves + wave) * 16u + slot] = __builtin_amdgcn_s_memrealtime();
    };
    sstamp(0);
    uint32_t iter = 0;
    uint32_t a_s = 0u, a_d = 0u, a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u, a_n = 0u;  // wave-uniform
    uint32_t a_k = 0u;  // the batch the counters belong to
    if (tid <= kAcc) s_acc[tid] = 0u;  // published by the prologue barrier

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
    };
    Set SS[D];
    uint4 pin[4];
    auto load_q = [&](uint32_t g, uint2& q) {
        const uint32_t k = batch_of(k_q, g);
        const uint32_t i = (g - SB.b[k].seg_start) * 64u + lane, n = SB.b[k].n;
        const uint32_t* off = SB.b[k].offsets;
        q = make_uint2(off[min(i, n)], off[min(i + 1u, n)]);
    };
    auto fetch = [&](Set& X, uint32_t g_h, uint32_t next_q) {  // X.q holds segment g_h's offsets
        load_headers1(frames_rsrc(batch_of(k_h, g_h)), X.q.x, X.h);
        X.c = make_uint2(vmov(X.q.x), vmov(X.q.y));
        load_q(next_q, X.q);
    };
    auto dropped_stores = [&]() {
        if constexpr ((FLAGS & kNoStore) == 0u) {
#pragma unroll
            for (int j = 0; j < ((FLAGS & kPartOut) ? 9 : 8); ++j)
                __builtin_amdgcn_raw_buffer_store_b32(0u, r_drop, kOob + 64u * j, 0, 0);
        }
    };
    auto load_parsed = [&](uint32_t sg) {
        const uint4* qq = reinterpret_cast<const uint4*>(P.parsed + min(sg * 64u + lane, P.n - 1u));
        pin[0] = qq[0];
        pin[1] = qq[1];
        pin[2] = qq[2];
        const uint2 t = *reinterpret_cast<const uint2*>(qq + 3);
        pin[3] = make_uint4(t.x, t.y, 0u, 0u);
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
        if (b == 0u && tid == 0u) *P.error_next = 0u;  // other parity's word, for the next launch
    }
    if constexpr (!PARSED) fetch(SS[0], sg, seg_of(Ln));
    dropped_stores();
    ws_tick();  // configuration in LDS (LDS-only barrier: the header loads stay in flight)
    sstamp(1);
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
            if constexpr ((FLAGS & kNoLookback) != 0u) {
                kk.cls = FB_CLASS_SESSION;
                kk.tcp = kk.v4 = true;
                kk.bad = false;
                const uint32_t hw[14] = {X.h.A.x, X.h.A.y, X.h.A.z, X.h.A.w, X.h.B.x, X.h.B.y, X.h.B.z, X.h.B.w, X.h.C.x, X.h.C.y, X.h.C.z, X.h.C.w, X.h.A.x ^ X.h.C.w, X.c.x};
    #pragma unroll
                for (int j = 0; j < 14; ++j) kk.w[j] = hw[j];
            } else if constexpr (!PARSED) {
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
            if (is_s) {
                unsigned long long* dd = stage + (size_t)__popcll(m_sess & lmask) * 7;
    #pragma unroll
                for (int w = 0; w < 7; ++w)
                    dd[w] = (unsigned long long)kk.w[2 * w] | ((unsigned long long)kk.w[2 * w + 1] << 32);
            }
            __builtin_amdgcn_wave_barrier();
            // prefetch: headers of this set's next segment (offsets already here), offsets of the
            // one after
            if constexpr (!PARSED) fetch(X, g_next, g_after);
            else load_parsed(g_next);
            if constexpr ((FLAGS & kNoStore) == 0u) {
            // stores: 4 x 16 B of session records, the 8-B tail, one DNS record, the count, the class
                const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<uint8_t*>(B.out) + (size_t)ls * kSegBytes, (short)0, (int)kSegBytes, 0x00020000);
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
                    __builtin_amdgcn_raw_buffer_store_b128(v, r_out, cc < body ? cc * 16u : kOob, 0, FB_ST_AUX);
                }
                {
                    const bool tail = (words & 1u) && lane == 0u;
                    const unsigned long long x = stage[words ? words - 1u : 0u];
                    const u32x2 v = {(uint32_t)x, (uint32_t)(x >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b64(v, r_out, tail ? (words - 1u) * 8u : kOob, 0, FB_ST_AUX);
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
                    __builtin_amdgcn_raw_buffer_store_b32(part_of(flow_hash_words(key), P.part_shift), r_part,
                                                          is_s ? (uint32_t)__popcll(m_sess & lmask) * 4u : kOob, 0, 0);
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
            sstamp(2u + min(iter++, 11u));
    };
    while (sg < nseg) {
        const uint32_t La = grab();
        const uint32_t g_next = seg_of(Ln);
        step(sg, SS[0], g_next, seg_of(La));
        Lc = Ln;
        Ln = La;
        sg = g_next;
    }
    sstamp(14);
    // ---- batch stats, no barrier and no partials read-back:
    // every wave adds its counters into LDS (per batch); the block's last wave (LDS arrival
    // count) adds the block's counters of every batch into that batch's 5 packed device words
    // [ticket:10 | hi:27 | lo:27] (one atomic per word, lanes 5k..5k+4 for batch k in parallel);
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
        if (arrived == (uint32_t)kSegWaves - 1u && lane < 5u * nb) {
            asm volatile("" ::: "memory");
            const uint32_t k = lane / 5u, j = lane - 5u * k;
            const unsigned long long lo = s_acc[k * 10u + 2u * j], hi = s_acc[k * 10u + 2u * j + 1u];
            unsigned long long* word = reinterpret_cast<unsigned long long*>(P.tick) + k * 8u + j;
            const unsigned long long add = (1ull << 54) | (hi << 27) | lo;
            const unsigned long long old = __hip_atomic_fetch_add(word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((old >> 54) == (unsigned long long)G - 1u) {
                const unsigned long long t = old + add, m27 = (1ull << 27) - 1ull;
                const unsigned long long f_lo = t & m27, f_hi = (t >> 27) & m27;
                __hip_atomic_store(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fb_batch_stats* S = SB.b[k].stats;
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
    sstamp(15);
}

hipError_t launch_parse_seg(const ParseParams& p, const SegBatches& sb, uint32_t grid, hipStream_t s) {
    if (p.parsed) hipLaunchKernelGGL((k_parse_seg<true>), dim3(grid), dim3(kSegThreads), 0, s, p, sb);
    else if (sb.count > 1u)
        hipLaunchKernelGGL((k_parse_seg<false, kFlagsProduct, true>), dim3(grid), dim3(kSegThreads), 0, s, p, sb);
    else if (p.rec_part)  // instantiated after the headline instance: its code placement is unchanged
        hipLaunchKernelGGL((k_parse_seg<false, kFlagsProduct | kPartOut>), dim3(grid), dim3(kSegThreads), 0, s, p, sb);
    else hipLaunchKernelGGL((k_parse_seg<false>), dim3(grid), dim3(kSegThreads), 0, s, p, sb);
    return hipGetLastError();
}
hipError_t occupancy_parse_seg(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (k_parse_seg<false>), kSegThreads, 0);
}
uint32_t parse_seg_block_threads() { return kSegThreads; }

hipError_t launch_parse_classify(const ParseParams& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((k_parse_ws<false>), dim3(grid), dim3(kWsThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_process_parsed(const ParseParams& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((k_parse_ws<true>), dim3(grid), dim3(kWsThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t occupancy_parse(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (k_parse_ws<false>), kWsThreads, 0);
}
uint32_t parse_unit_frames() { return kWsUnit; }
uint32_t parse_block_waves() { return kWsThreads / 64; }

}  // namespace fbk
