// fb_parse.hip -- gfx950 parse + classify kernel (persistent, wave-level lag-1 pipeline).
//
// One wavefront lane per frame.  Replaces, per frame:
//   parse_packet_pcap                 src/packets.rs:603-802 (pnet_packet 0.35.0 decode)
//   service-port direction + key      src/packets.rs:232-311 (get_name_from_port, port_vulns.rs:213)
//   is_originator                     src/packets.rs:316-319
//   Local/Global session filter       src/packets.rs:321-327, sessions.rs:660-672, ip.rs:199-242
//   PACKET_STATS pre-filter counters  src/packets.rs:211-227
//   map_tcp_flags (history char)      src/packets.rs:561-601
//
// Output is stream-compacted in packet order (SESSION records, DNS side records), so each tile
// needs the global count of records emitted before it: a decoupled look-back.  Measured on a
// one-tile-per-block kernel (C2, 1M x 64 B): 45 us, 14 us of it look-back waits, because all
// resident blocks load, then all wait, then all store, with HBM idle during the wait.
//
// Here every WAVE is an independent agent with no block barrier in its loop:
//   grid = co-resident blocks of 4 waves; wave w (of W) owns wave-tiles w, w+W, w+2W, ...
//   (a wave-tile = 64*R frames; static ownership, no ticket atomics: every tile a look-back
//   waits on belongs to a running wave because the grid never exceeds residency).
//   iteration: wait headers(cur) -> decode/classify into registers -> publish cur's count
//              -> probe the look-back words of PREV (the wave's previous tile, classified one
//                 iteration ago, so its predecessors are normally published by now)
//              -> issue header loads of next and offset loads of the tile after (younger than
//                 the probes, so the probes do not wait for them)
//              -> finish the look-back (all not-ready lanes re-poll together) -> store prev's
//                 records with coalesced 16-B stores from the wave's LDS stage -> stage cur.
//   HBM sees one tile of header loads per wave in flight across the look-back and the stores.
//
// Loads: four unaligned 16-B header loads per frame at frame offsets 10, 26, 42 (+ one dword at
// 66 for IPv6/TCP) so every decoder field sits at a fixed dword/byte position; buffer loads are
// range-checked against frames_bytes, so nothing reads past the batch.
#include "fb_internal.h"

namespace fbk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

// be16 of bytes 0,1 / 2,3 of a little-endian dword.
__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t w) { return ((w >> 8) & 0xff00u) | (w >> 24); }
__device__ __forceinline__ uint32_t bswap(uint32_t w) { return __builtin_bswap32(w); }

__device__ __forceinline__ uint32_t svc(const uint32_t* bm, uint32_t p) { return (bm[p >> 5] >> (p & 31)) & 1u; }

// is_lan_ip, src/ip.rs:55-156, 199-242.
__device__ __forceinline__ bool lan_v4(uint32_t v) {
    uint32_t a = v >> 24, b = (v >> 16) & 0xffu;
    return v == 0u || v == 0xffffffffu || a == 127u || (v >> 28) == 0xEu || (v >> 16) == 0xA9FEu ||
           a == 10u || (a == 172u && b >= 16u && b <= 31u) || (v >> 16) == 0xC0A8u;
}
__device__ __forceinline__ bool lan_v6(const DevConfig* c, const uint32_t w[4]) {
    uint32_t s0 = w[0] >> 16;
    if ((w[0] | w[1] | w[2] | w[3]) == 0u) return true;                       // ::
    if ((w[0] | w[1] | w[2]) == 0u && w[3] == 1u) return true;                // ::1
    if ((s0 & 0xffc0u) == 0xfe80u || (s0 & 0xff00u) == 0xff00u || (s0 & 0xfe00u) == 0xfc00u)
        return true;                                                          // fe80::/10 ff00::/8 fc00::/7
    const uint32_t nl = c->n_lan_v6;                                          // uniform loop
    for (uint32_t i = 0; i < nl; ++i) {
        const LanV6& e = c->lan_v6[i];
        if ((w[0] & e.mask[0]) == e.net[0] && (w[1] & e.mask[1]) == e.net[1] &&
            (w[2] & e.mask[2]) == e.net[2] && (w[3] & e.mask[3]) == e.net[3])
            return true;
    }
    return false;
}
__device__ __forceinline__ bool own_ip(const DevConfig* c, uint32_t fam, const uint32_t w[4]) {
    const uint32_t no = c->n_own;
    bool hit = false;
    for (uint32_t i = 0; i < no; ++i) {
        const fb_ip& o = c->own[i];
        hit |= o.family == fam && o.addr[0] == w[0] && o.addr[1] == w[1] && o.addr[2] == w[2] &&
               o.addr[3] == w[3];
    }
    return hit;
}

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

struct Hdr {
    u32x4 A, B, C;  // f[10..25] f[26..41] f[42..57]
    uint32_t Dz;    // f[66..69] (IPv6 TCP data offset + flags)
};

struct Pkt {
    uint32_t cls;         // fb_class after filtering
    uint32_t w[14];       // the fb_pkt_out record (SESSION) / dns fields (DNS)
    bool tcp, v4, bad;    // stats bits (valid when session or filtered)
};

// ---- process_parsed_packet, src/packets.rs:202-327, for one SessionPacketData -------------
// (raw 5-tuple src/dst/ports as parsed, L4 payload length, IP length, TCP flags if any) ->
// canonical session key, originator, local/global filter, history char; k.cls = SESSION or
// FILTERED.  Shared by the frame path (process_frame) and the parsed-packet path.
__device__ __forceinline__ void classify_session(const DevConfig* cfg, const uint32_t* bm, uint32_t proto,
                                                 uint32_t fam, const uint32_t (&src)[4], const uint32_t (&dst)[4],
                                                 uint32_t sport, uint32_t dport, uint32_t hasf, uint32_t flags,
                                                 uint32_t plen, uint32_t iplen, uint32_t idx, Pkt& k) {
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
    const bool lan_s = fam == 2u ? lan_v4(ks[0]) : lan_v6(cfg, ks);
    const bool lan_d = fam == 2u ? lan_v4(kd[0]) : lan_v6(cfg, kd);
    uint32_t meta = hasf;
    meta |= swap ? FB_META_SWAP : 0u;
    meta |= orig ? FB_META_ORIGINATOR : 0u;
    meta |= lan_s ? FB_META_LOCAL_SRC : 0u;
    meta |= lan_d ? FB_META_LOCAL_DST : 0u;
    meta |= own_ip(cfg, fam, ks) ? FB_META_SELF_SRC : 0u;
    meta |= own_ip(cfg, fam, kd) ? FB_META_SELF_DST : 0u;
    meta |= svc(bm, kport_d) ? FB_META_DST_SERVICE : 0u;
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
                                              const uint32_t* bm, const Hdr& h, uint32_t o0, uint32_t o1,
                                              uint32_t fbytes, uint32_t idx, Pkt& k) {
    k.cls = FB_CLASS_DROP;
    k.tcp = false;
    k.v4 = false;
    const bool okoff = o1 >= o0 && o1 <= fbytes;
    k.bad = !okoff;
    const uint32_t L = okoff ? o1 - o0 : 0u;
    const u32x4 A = h.A, B = h.B, C = h.C;
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
        d3 = h.Dz;                                           // f[66..69]
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

    classify_session(cfg, bm, proto, fam, src, dst, sport, dport, hasf, flags, plen, iplen, idx, k);
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
// Ablation switches (tools/ubench_parse.hip); the product instantiates kFlagsProduct.
constexpr uint32_t kFlagsProduct = 0u;
constexpr uint32_t kNoLookback = 1u;  // base offsets = tile start (wrong output, timing only)
constexpr uint32_t kNoStore = 2u;     // no record / dns stores (timing only)
constexpr uint32_t kStamps = 4u;      // per-tile s_memrealtime stamps + poll counts into P.dbg
// dbg layout per tile t: [0] classified, [1] look-back issued, [2] look-back done, [3] spins

// ---- look-back ----------------------------------------------------------------------------
// One status word per unit, epoch-tagged: [epoch:8 | INC:1 | n_dns:27 | n_session:28].
//   published twice by the unit's look-back wave with plain sc1 stores (no atomics, no shared
//   accumulator line that every block hammers): AGG (its own count) right after classification,
//   INC (its inclusive prefix) once its look-back is done.
// Look-back of unit u: read predecessors u-1, u-2, ... in windows of 256 (4 words per lane, one
// memory round trip), stop at the nearest INC; every word up to it must be published (AGG or
// INC of this epoch).  Not-ready words are re-polled by their lanes together with exponential
// back-off, so a wait costs one round trip per readiness event, not one per word.
constexpr unsigned long long kIncBit = 1ull << 55;
constexpr unsigned long long kCnt28 = (1ull << 28) - 1ull;
__device__ __forceinline__ unsigned long long st_counts(unsigned long long w) {
    return (w & kCnt28) | (((w >> 28) & ((1ull << 27) - 1ull)) << 28);
}
__device__ __forceinline__ unsigned long long st_pack(uint32_t ep, bool inc, unsigned long long c) {
    return ((unsigned long long)ep << 56) | (inc ? kIncBit : 0ull) | (c & kCnt28) |
           (((c >> 28) & ((1ull << 27) - 1ull)) << 28);
}

template <uint32_t FLAGS, int NW = 4>
__device__ unsigned long long lookback_unit(const ParseParams& P, uint32_t u, uint32_t& spins) {
    constexpr int WIN = 64 * NW;  // predecessors probed per round trip
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t ep = P.epoch;
    // sc1 buffer loads (aux 16): L1-bypassing like the agent-scope atomic loads, 32-bit offsets,
    // and out-of-range offsets (negative indices) read as 0 = "not published".
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.tagg, (short)0, (int)(u * 8u), 0x00020000);
    auto word = [&](int idx) {
        const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rt, (uint32_t)idx * 8u, 0, 16);
        return (unsigned long long)x.x | ((unsigned long long)x.y << 32);
    };
    unsigned long long pre = 0ull;
    int lo = (int)u - WIN;  // window = [lo, lo + WIN), lane l of chunk k reads lo + 64k + l
    spins = 0u;
    for (;;) {
        unsigned long long v[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) v[k] = word(lo + 64 * k + (int)lane);
        for (;;) {
            // nearest published inclusive prefix = the highest index carrying INC
            int near = -1;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const int idx = lo + 64 * k + (int)lane;
                const unsigned long long im = __ballot(idx >= 0 && tag_of(v[k]) == ep && (v[k] & kIncBit));
                if (im) near = lo + 64 * k + (63 - __clzll((long long)im));
            }
            const int floor_idx = near >= 0 ? near : (lo > 0 ? lo : 0);  // words below are not needed
            bool ready = true;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const int idx = lo + 64 * k + (int)lane;
                ready &= idx < floor_idx || tag_of(v[k]) == ep;
            }
            if (__ballot(!ready) == 0ull) {
                unsigned long long sum = 0ull;
#pragma unroll
                for (int k = 0; k < NW; ++k) {
                    const int idx = lo + 64 * k + (int)lane;
                    sum += idx >= floor_idx ? st_counts(v[k]) : 0ull;
                }
                pre += wave_sum64(sum);
                if (near >= 0 || lo <= 0) return pre;
                break;
            }
            if (++spins > (1u << 16)) { if (lane == 0u) atomicOr(P.error, 1u); return pre; }
            // exponential back-off: every poll is a memory-side read
            for (uint32_t z = 0; z < min(spins, 6u); ++z) __builtin_amdgcn_s_sleep(8);
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const int idx = lo + 64 * k + (int)lane;
                if (idx >= floor_idx && tag_of(v[k]) != ep) v[k] = word(idx);
            }
        }
        lo -= WIN;  // no INC in this window: every word was an aggregate, continue below it
    }
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

template <int V>
struct IC {
    static constexpr int value = V;
};

__device__ __forceinline__ void load_headers1(__amdgpu_buffer_rsrc_t rs, uint32_t o, Hdr& h) {
    h.A = ld16(rs, o + 10u);
    h.B = ld16(rs, o + 26u);
    h.C = ld16(rs, o + 42u);
    h.Dz = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 66u, 0, 0);
}

// One look-back unit = one block-round: kWaves waves x U wave-tiles x 64 frames.  Block b
// (of G co-resident blocks) owns units b, b+G, b+2G, ...; inside a unit, wave w owns the
// contiguous frames [w*U*64, (w+1)*U*64), so packet order = (wave, tile, lane).  Per unit:
//   1. every wave issues the offsets of its U tiles, then all 4U header loads (U*64 frames of
//      loads in flight per wave)
//   2. every wave classifies and stages its SESSION records, compacted, in its own LDS region
//      (records do not stay live in VGPRs across the look-back); counts -> LDS     | barrier
//   3. wave 0 publishes the unit's count and runs the look-back: ONE participant per block
//      (a few hundred per launch) keeps the polled words cold; lanes poll together with
//      exponential back-off                                                          | barrier
//   4. every wave copies its LDS region to its place in the output with coalesced 16-B
//      stores; DNS records straight from registers
template <int U, uint32_t FLAGS, bool PARSED = false>
__global__ __launch_bounds__(kThreads) void k_parse_block(const ParseParams P) {
    constexpr uint32_t kWaves = kThreads / 64;
    constexpr uint32_t WF = 64u * U;          // frames per wave per unit
    constexpr uint32_t UF = WF * kWaves;      // frames per unit
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t G = gridDim.x, T = P.num_tiles;  // T = units
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;

    __shared__ DevConfig s_cfg;                                  // service bitmap + tables
    __shared__ unsigned long long s_stage_all[kWaves][WF * 7];  // per-wave compacted records
    __shared__ uint32_t s_cnt[kWaves][4];                        // sessions, dns, filtered|tcp, v4|bad
    __shared__ unsigned long long s_excl;
    unsigned long long* s_stage = s_stage_all[wave];
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        uint4* dst = reinterpret_cast<uint4*>(&s_cfg);
        for (uint32_t q = tid; q < sizeof(DevConfig) / 16; q += kThreads) dst[q] = src[q];
        // Zero the other parity's error word for the next launch (the previous launch, which
        // used it, has completed: launches on one context are stream-ordered).
        if (blockIdx.x == 0u && tid == 0u) *P.error_next = 0u;
    }
    __syncthreads();
    const DevConfig* cfg = &s_cfg;

    const unsigned long long lmask = (1ull << lane) - 1ull;
    uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;  // pre-filter counters (block, wave 0 keeps them)

    for (uint32_t u = blockIdx.x; u < T; u += G) {
        const uint32_t f0 = u * UF + wave * WF;  // first frame of this wave
        // ---- 1. loads -----------------------------------------------------------------------
        uint2 o[U];
        Hdr h[U];
        uint4 pin[U][4];  // PARSED: one fb_parsed_pkt (56 B) per lane
        if constexpr (!PARSED) {
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = f0 + r * 64u + lane;
                o[r] = make_uint2(P.offsets[min(i, P.n)], P.offsets[min(i + 1u, P.n)]);  // n+1 entries
            }
#pragma unroll
            for (int r = 0; r < U; ++r) load_headers1(rs, o[r].x, h[r]);
        } else {
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = min(f0 + r * 64u + lane, P.n - 1u);  // n >= 1 here
                const uint4* q = reinterpret_cast<const uint4*>(P.parsed + i);
                pin[r][0] = q[0];
                pin[r][1] = q[1];
                pin[r][2] = q[2];
                const uint2 t = *reinterpret_cast<const uint2*>(q + 3);
                pin[r][3] = make_uint4(t.x, t.y, 0u, 0u);
            }
        }
        // ---- 2. classify + stage ----------------------------------------------------------------
        unsigned long long m_dns[U];
        uint4 dnsw[U];
        uint32_t cs = 0u, cd = 0u, wf = 0u, wt = 0u, w4 = 0u, wb = 0u;
#pragma unroll
        for (int r = 0; r < U; ++r) {
            const uint32_t i = f0 + r * 64u + lane;
            const bool valid = i < P.n;
            Pkt k;
            if constexpr (!PARSED) {
                process_frame(rs, cfg, cfg->service_bitmap, h[r], valid ? o[r].x : 1u, valid ? o[r].y : 0u,
                              P.frames_bytes, i, k);
            } else {
                // fb_parsed_pkt: session_key words 0..9, then lengths, flags, pkt_index
                const uint4 a = pin[r][0], b = pin[r][1], c = pin[r][2], d = pin[r][3];
                const uint32_t src[4] = {a.x, a.y, a.z, a.w}, dst[4] = {b.x, b.y, b.z, b.w};
                const uint32_t proto = c.y & 0xffu, fam = (c.y >> 8) & 0xffu;
                k.bad = false;
                k.cls = FB_CLASS_DROP;
                k.tcp = k.v4 = false;
                if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                    classify_session(cfg, cfg->service_bitmap, proto, fam, src, dst, c.x & 0xffffu, c.x >> 16,
                                     (d.x >> 8) & 1u, d.x & 0xffu, c.z, c.w, d.y, k);
            }
            const bool is_s = valid && k.cls == FB_CLASS_SESSION;
            const bool is_d = valid && k.cls == FB_CLASS_DNS;
            const bool is_f = valid && k.cls == FB_CLASS_FILTERED;
            const bool counted = is_s || is_f;
            const unsigned long long m_sess = __ballot(is_s);
            m_dns[r] = __ballot(is_d);
            dnsw[r] = make_uint4(k.w[0], k.w[1], k.w[2], k.w[3]);
            if (is_s) {
                unsigned long long* d = s_stage + (size_t)(cs + __popcll(m_sess & lmask)) * 7;
#pragma unroll
                for (int w = 0; w < 7; ++w)
                    d[w] = (unsigned long long)k.w[2 * w] | ((unsigned long long)k.w[2 * w + 1] << 32);
            }
            cs += (uint32_t)__popcll(m_sess);
            cd += (uint32_t)__popcll(m_dns[r]);
            wf += __popcll(__ballot(is_f));
            wt += __popcll(__ballot(counted && k.tcp));
            w4 += __popcll(__ballot(counted && k.v4));
            wb += __popcll(__ballot(valid && k.bad));
            if (valid && P.cls) P.cls[i] = (uint8_t)k.cls;
        }
        if (lane == 0u) {
            s_cnt[wave][0] = cs;
            s_cnt[wave][1] = cd;
            s_cnt[wave][2] = wf | (wt << 16);
            s_cnt[wave][3] = w4 | (wb << 16);
        }
        __syncthreads();  // counts of every wave
        // ---- 3. publish + look-back (wave 0) --------------------------------------------------
        if (wave == 0u) {
            uint32_t bs = 0u, bd = 0u;
#pragma unroll
            for (uint32_t w = 0; w < kWaves; ++w) {
                bs += s_cnt[w][0];
                bd += s_cnt[w][1];
                a_f += s_cnt[w][2] & 0xFFFFu;
                a_t += s_cnt[w][2] >> 16;
                a_4 += s_cnt[w][3] & 0xFFFFu;
                a_b += s_cnt[w][3] >> 16;
            }
            const unsigned long long agg = (unsigned long long)bs | ((unsigned long long)bd << 28);
            if constexpr ((FLAGS & kStamps) != 0u)
                if (lane == 0u) P.dbg[4ull * u] = __builtin_amdgcn_s_memrealtime();
            unsigned long long excl;
            if (FLAGS & kNoLookback) {
                excl = (unsigned long long)u * UF;
            } else {
                if (lane == 0u) ast(P.tagg + u, st_pack(ep, false, agg));
                uint32_t spins;
                excl = lookback_unit<FLAGS>(P, u, spins);
                if (lane == 0u) ast(P.tagg + u, st_pack(ep, true, excl + agg));
                if constexpr ((FLAGS & kStamps) != 0u)
                    if (lane == 0u) {
                        P.dbg[4ull * u + 2] = __builtin_amdgcn_s_memrealtime();
                        P.dbg[4ull * u + 3] = spins;
                    }
            }
            if (lane == 0u) s_excl = excl;
            if (u == T - 1u && P.stats && !(FLAGS & kNoLookback)) {
                // the last unit's owner: own counters first (this is the block's last unit)
                if (lane == 0u) {
                    ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
                    ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
                }
                write_batch_stats(P, excl + agg, G);
            }
        }
        __syncthreads();  // s_excl
        // ---- 4. stores ---------------------------------------------------------------------------
        if (!(FLAGS & kNoStore)) {
            const unsigned long long bex = s_excl;
            uint32_t base_s = (uint32_t)(bex & ((1ull << 28) - 1ull));
            uint32_t base_d = (uint32_t)(bex >> 28);
            for (uint32_t w = 0; w < wave; ++w) {
                base_s += s_cnt[w][0];
                base_d += s_cnt[w][1];
            }
            if (P.out && cs) {
                // [base_s*56, (base_s+cs)*56) is 8-B aligned: 16-B aligned body + 8-B head/tail
                unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7;
                const uint32_t units = cs * 7, head = base_s & 1u, body = (units - head) >> 1;
                if (head && lane == 0u) g8[0] = s_stage[0];
                uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                for (uint32_t c = lane; c < body; c += 64u) {
                    const unsigned long long x = s_stage[head + 2 * c], y = s_stage[head + 2 * c + 1];
                    g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                }
                if (lane == 0u && head + 2 * body < units) g8[units - 1] = s_stage[units - 1];
            }
            if (P.dns) {
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    if ((m_dns[r] >> lane) & 1ull) {
                        fb_dns_out d;
                        d.pkt_index = dnsw[r].x;
                        d.payload_offset = dnsw[r].y;
                        d.payload_length = dnsw[r].z;
                        d.protocol = (uint8_t)(dnsw[r].w & 0xffu);
                        d.family = (uint8_t)(dnsw[r].w >> 8);
                        d.reserved = 0;
                        P.dns[base_d + __popcll(m_dns[r] & lmask)] = d;
                    }
                    base_d += (uint32_t)__popcll(m_dns[r]);
                }
            }
        }
        __syncthreads();  // s_cnt / s_excl / stage reuse by the next unit
    }
    // every block publishes its pre-filter counters (the last unit's owner did so above)
    const bool owner_last = T > 0u && (T - 1u) % G == blockIdx.x;
    if (!owner_last && tid == 0u && !(FLAGS & kNoLookback)) {
        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
    }
}

hipError_t launch_parse_classify(const ParseParams& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((k_parse_block<kUnitTiles, kFlagsProduct>), dim3(grid), dim3(kThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_process_parsed(const ParseParams& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((k_parse_block<kUnitTiles, kFlagsProduct, true>), dim3(grid), dim3(kThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t occupancy_parse(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (k_parse_block<kUnitTiles, kFlagsProduct>),
                                                        kThreads, 0);
}

}  // namespace fbk
