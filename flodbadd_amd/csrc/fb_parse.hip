// fb_parse.hip -- gfx950 parse + classify kernel.
//
// One wavefront lane per frame.  Replaces, per frame:
//   parse_packet_pcap                 src/packets.rs:603-802 (pnet_packet 0.35.0 decode)
//   service-port direction + key      src/packets.rs:232-311 (get_name_from_port, port_vulns.rs:213)
//   is_originator                     src/packets.rs:316-319
//   Local/Global session filter       src/packets.rs:321-327, sessions.rs:660-672, ip.rs:199-242
//   PACKET_STATS pre-filter counters  src/packets.rs:211-227
//   map_tcp_flags (history char)      src/packets.rs:561-601
//
// Memory plan (HBM-bound integer/byte work, no MFMA):
//   * offsets: one coalesced u32 per lane (+ next lane's via DPP shuffle).
//   * frame header: four unaligned 16-B buffer loads per lane at frame offsets 10, 26, 42, 58
//     (gfx950 runs in unaligned-access mode).  Offsets are chosen so every field the decoder
//     needs sits at a fixed dword/byte position:  A=f[10..25] B=f[26..41] C=f[42..57]
//     D=f[58..73].  Only an IPv4 header with options needs a fifth (dependent) load.
//     Buffer loads are range-checked against frames_bytes: no read past the batch.
//   * records: compacted in packet order by wave ballot + mbcnt, a per-block prefix over
//     (round, wave) and a decoupled look-back across tiles (blockIdx order); one 56-B record
//     per emitted packet.  No same-address atomics anywhere (they serialise at ~12 ns each).
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

__device__ __forceinline__ uint32_t svc(const DevConfig* c, uint32_t p) {
    return (c->service_bitmap[p >> 5] >> (p & 31)) & 1u;
}

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

struct Pkt {
    uint32_t cls;         // fb_class after filtering
    uint32_t w[14];       // the fb_pkt_out record (SESSION) / dns fields (DNS)
    bool tcp, v4, bad;    // stats bits (valid when session or filtered)
};

// Decode + classify one frame.  All byte reads come from the four header vectors; a field is
// only used when the pnet length rules guarantee it lies inside the frame's caplen.
__device__ __forceinline__ void process_frame(__amdgpu_buffer_rsrc_t r, const DevConfig* cfg,
                                              uint32_t o0, uint32_t o1, uint32_t fbytes,
                                              uint32_t idx, Pkt& k) {
    k.cls = FB_CLASS_DROP;
    k.tcp = false;
    k.v4 = false;
    const bool okoff = o1 >= o0 && o1 <= fbytes;
    k.bad = !okoff;
    const uint32_t L = okoff ? o1 - o0 : 0u;
    const u32x4 A = ld16(r, o0 + 10u), B = ld16(r, o0 + 26u), C = ld16(r, o0 + 42u),
                D = ld16(r, o0 + 58u);
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
        d3 = D.z;                                            // f[66..69]
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

    // ---- process_parsed_packet, src/packets.rs:202-327 -------------------------------------
    k.tcp = proto == 6u;
    k.v4 = fam == 2u;
    const uint32_t S = svc(cfg, sport), Dsv = svc(cfg, dport);
    bool swap;
    if (S && !Dsv) {
        swap = true;
    } else if (S && Dsv) {
        if (hasf && (flags & 0x02u) && !(flags & 0x10u)) swap = false;       // SYN
        else if (hasf && (flags & 0x02u) && (flags & 0x10u)) swap = true;    // SYN+ACK
        else swap = sport < dport;                                          // port tiebreak
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
    meta |= svc(cfg, kport_d) ? FB_META_DST_SERVICE : 0u;
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

__device__ __forceinline__ unsigned long long ld_status(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Publish one 4-word status set: payload words first, drained, then the epoch-tagged word 0
// (MI355X_MICROARCH.md "Valid forms": 8-B agent atomics on both sides + vmcnt(0) before flag).
__device__ __forceinline__ void publish(unsigned long long* s, const unsigned long long v[4],
                                        uint32_t epoch) {
    st_status(s + 1, v[1]);
    st_status(s + 2, v[2]);
    st_status(s + 3, v[3]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_status(s + 0, ((unsigned long long)epoch << 32) | (v[0] & 0xffffffffull));
}

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(kThreads) void k_parse_classify(const ParseParams P) {
    const uint32_t tile = blockIdx.x;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const DevConfig* cfg = P.cfg;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);

    __shared__ uint32_t s_cnt[kRounds][4][2];   // per (round, wave): sessions, dns
    __shared__ uint32_t s_aux[kRounds][4][4];   // filtered, tcp, ipv4, bad
    __shared__ unsigned long long s_excl[4];

    Pkt k[kRounds];
    unsigned long long m_sess[kRounds], m_dns[kRounds];
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
        const uint32_t i = tile * kTile + rd * kThreads + tid;
        const bool valid = i < P.n;
        // offsets has n+1 entries: lane i reads offsets[min(i, n)], so the last frame's end
        // offset arrives from the next lane; lane 63 reads its own.
        uint32_t o0 = P.offsets[min(i, P.n)];
        uint32_t o1 = __shfl_down(o0, 1, 64);
        if (lane == 63u && valid) o1 = P.offsets[i + 1];
        if (!valid) { o0 = 1u; o1 = 0u; }   // forces DROP, no stats (masked below)
        process_frame(rs, cfg, o0, o1, P.frames_bytes, i, k[rd]);
        const bool is_s = valid && k[rd].cls == FB_CLASS_SESSION;
        const bool is_d = valid && k[rd].cls == FB_CLASS_DNS;
        const bool is_f = valid && k[rd].cls == FB_CLASS_FILTERED;
        const bool counted = is_s || is_f;
        m_sess[rd] = __ballot(is_s);
        m_dns[rd] = __ballot(is_d);
        const unsigned long long m_f = __ballot(is_f);
        const unsigned long long m_t = __ballot(counted && k[rd].tcp);
        const unsigned long long m_4 = __ballot(counted && k[rd].v4);
        const unsigned long long m_b = __ballot(valid && k[rd].bad);
        if (lane == 0u) {
            s_cnt[rd][wave][0] = __popcll(m_sess[rd]);
            s_cnt[rd][wave][1] = __popcll(m_dns[rd]);
            s_aux[rd][wave][0] = __popcll(m_f);
            s_aux[rd][wave][1] = __popcll(m_t);
            s_aux[rd][wave][2] = __popcll(m_4);
            s_aux[rd][wave][3] = __popcll(m_b);
        }
        if (valid && P.cls) P.cls[i] = (uint8_t)k[rd].cls;
    }
    __syncthreads();

    // ---- tile aggregate + decoupled look-back (wave 0) ----------------------------------
    if (wave == 0u) {
        unsigned long long agg[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll
        for (int rd = 0; rd < kRounds; ++rd)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                agg[0] += s_cnt[rd][w][0];
                agg[1] += ((unsigned long long)s_cnt[rd][w][1] << 32) | s_aux[rd][w][0];
                agg[2] += ((unsigned long long)s_aux[rd][w][1] << 32) | s_aux[rd][w][2];
                agg[3] += (unsigned long long)s_aux[rd][w][3] << 32;
            }
        unsigned long long* st_agg = P.status + (size_t)tile * kStatusWords;
        unsigned long long* st_inc = st_agg + 4;
        unsigned long long ex[4] = {0ull, 0ull, 0ull, 0ull};
        const unsigned long long ep = (unsigned long long)P.epoch << 32;
        if (tile != 0u) {
            if (lane == 0u) publish(st_agg, agg, P.epoch);
            long pred = (long)tile - 1;
            bool spin_fail = false;
            for (;;) {
                const long t = pred - (long)lane;  // lane 0 = nearest predecessor
                bool virt = t < 0;                 // before tile 0: an empty inclusive prefix
                unsigned long long vi = 0ull, va = 0ull;
                bool inc_ok = virt, agg_ok = false;
                uint32_t spins = 0u;
                for (;;) {
                    if (!virt && !inc_ok && !agg_ok) {
                        const unsigned long long* s = P.status + (size_t)t * kStatusWords;
                        vi = ld_status(s + 4);
                        inc_ok = (vi & 0xffffffff00000000ull) == ep;
                        if (!inc_ok) {
                            va = ld_status(s);
                            agg_ok = (va & 0xffffffff00000000ull) == ep;
                        }
                    }
                    if (__all(inc_ok || agg_ok)) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 24)) { spin_fail = true; break; }
                }
                if (spin_fail) break;
                const unsigned long long pm = __ballot(inc_ok);
                const uint32_t first = pm ? (uint32_t)(__ffsll((long long)pm) - 1) : 64u;
                unsigned long long c[4] = {0ull, 0ull, 0ull, 0ull};
                if (lane <= first && !virt) {
                    const unsigned long long* s = P.status + (size_t)t * kStatusWords + (lane == first ? 4 : 0);
                    c[0] = (lane == first ? vi : va) & 0xffffffffull;
                    c[1] = ld_status(s + 1);
                    c[2] = ld_status(s + 2);
                    c[3] = ld_status(s + 3);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) ex[j] += wave_sum64(c[j]);
                if (pm) break;
                pred -= 64;
            }
            if (spin_fail && lane == 0u) atomicOr(P.error, 1u);
        }
        unsigned long long inc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) inc[j] = ex[j] + agg[j];
        if (lane == 0u) {
            publish(st_inc, inc, P.epoch);
#pragma unroll
            for (int j = 0; j < 4; ++j) s_excl[j] = ex[j];
            if (tile == P.num_tiles - 1u && P.stats) {   // totals of the whole batch
                fb_batch_stats* S = P.stats;
                const unsigned long long ns = inc[0] & 0xffffffffull, nd = inc[1] >> 32,
                                         nf = inc[1] & 0xffffffffull, nt = inc[2] >> 32,
                                         n4 = inc[2] & 0xffffffffull, nb = inc[3] >> 32;
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
                S->error = 0ull;
                S->reserved[0] = S->reserved[1] = S->reserved[2] = 0ull;
            }
        }
    }
    __syncthreads();

    // ---- scatter records in packet order ---------------------------------------------------
    uint32_t base_s = (uint32_t)(s_excl[0] & 0xffffffffull);
    uint32_t base_d = (uint32_t)(s_excl[1] >> 32);
    const unsigned long long lmask = (1ull << lane) - 1ull;
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
        uint32_t ps = base_s, pd = base_d;
        for (uint32_t w = 0; w < wave; ++w) {
            ps += s_cnt[rd][w][0];
            pd += s_cnt[rd][w][1];
        }
        if (P.out && ((m_sess[rd] >> lane) & 1ull)) {
            const uint32_t pos = ps + __popcll(m_sess[rd] & lmask);
            uint32_t* o = reinterpret_cast<uint32_t*>(P.out + pos);
#pragma unroll
            for (int j = 0; j < 14; j += 2)
                *reinterpret_cast<uint2*>(o + j) = make_uint2(k[rd].w[j], k[rd].w[j + 1]);
        }
        if (P.dns && ((m_dns[rd] >> lane) & 1ull)) {
            const uint32_t pos = pd + __popcll(m_dns[rd] & lmask);
            *reinterpret_cast<uint4*>(P.dns + pos) = make_uint4(k[rd].w[0], k[rd].w[1], k[rd].w[2], k[rd].w[3]);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            base_s += s_cnt[rd][w][0];
            base_d += s_cnt[rd][w][1];
        }
    }
}

hipError_t launch_parse_classify(const ParseParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_parse_classify, dim3(p.num_tiles), dim3(kThreads), 0, s, p);
    return hipGetLastError();
}

}  // namespace fbk
