// fb_dns.hip -- DNS divert parse.
//
// The reference hands every port-53 payload to DnsPacketProcessor::process_dns_packet
// (src/dns.rs:35-99), which runs dns_parser::Packet::parse (dns-parser 0.8.0, a git dependency
// absent from the reference mount: its rules are restated here from its published source and are
// "parity unpinned") and then, for a query, keeps (id -> first question's name)
// unless it is a reverse lookup, and for a response, maps every A / AAAA answer to that name.
// k_dns_parse does the parse, one lane per DNS message (the byte-serial work); the bookkeeping
// is a few map operations per message and stays on the host, in order.
//
// Parse rules (dns-parser 0.8.0): header 12 bytes; every question (name, known QTYPE, known
// QCLASS), every answer / authority / additional record (name, known TYPE, known CLASS except
// for OPT, rdlen within the message, RDATA checks for A / AAAA / CNAME / NS / PTR / MX / SRV /
// SOA / TXT) must parse or the whole packet is rejected; an additional record starting
// 00 00 29 is the EDNS OPT record (a second one is an error).  Names: labels of <= 63 bytes that
// are ASCII, compression pointers that must point strictly before every earlier pointer target
// of the same name (so no loops), and the name's byte length in place (up to and including the
// first pointer).
#include "fb_internal.h"

namespace fbk {

// Bytes of one message.  The parse is a chain of dependent byte reads (label lengths, pointers),
// so serving it from LDS instead of HBM is what sets its speed.  MsgLds: the whole message is in
// the wavefront's LDS copy (row = the dword holding its first byte, mis = that byte's offset in
// it).  MsgMixed: the first `staged` bytes from LDS, the rest from HBM by a range-checked buffer
// load (a plain pointer there lets the compiler fold both sides into one generic flat load per
// byte, which waits on both counters).  ascii(a, b): no byte of [a, b) has its top bit set.
struct MsgLds {
    const uint32_t* row;
    uint32_t mis;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        return reinterpret_cast<const uint8_t*>(row)[i + mis];
    }
    __device__ __forceinline__ bool ascii(uint32_t a, uint32_t b) const {  // a dword per step
        const uint32_t p0 = a + mis, p1 = b + mis;
        uint32_t bad = 0u;
        for (uint32_t q = p0 & ~3u; q < p1; q += 4u) {
            uint32_t m = 0x80808080u;
            if (q < p0) m &= 0xFFFFFFFFu << (8u * (p0 - q));
            if (q + 4u > p1) m &= 0xFFFFFFFFu >> (8u * (q + 4u - p1));
            bad |= row[q >> 2] & m;
        }
        return bad == 0u;
    }
};
struct MsgMixed {
    const uint8_t* s;          // LDS copy of bytes [0, staged)
    __amdgpu_buffer_rsrc_t g;  // the frame buffer
    uint32_t off;              // the message's byte offset in it
    uint32_t staged;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        return i < staged ? (uint32_t)s[i] : (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(g, off + i, 0, 0);
    }
    __device__ __forceinline__ bool ascii(uint32_t a, uint32_t b) const {
        for (uint32_t k = a; k < b; ++k)
            if ((*this)(k) >= 0x80u) return false;
        return true;
    }
};

template <class M>
__device__ __forceinline__ uint32_t be16at(const M& m, uint32_t i) { return (m(i) << 8) | m(i + 1u); }

// Name::scan over the slice m[start..limit) with pointers into m[0..len); *blen = byte_len().
template <class M>
__device__ uint32_t dns_name_scan(const M& m, uint32_t len, uint32_t start, uint32_t limit, uint32_t* blen) {
    uint32_t base = start, lim = limit, pos = 0u;
    if (lim <= base) return FB_DNS_UNEXPECTED_EOF;
    uint32_t largest = len;
    int32_t ret = -1;
    uint32_t byte = m(base);
    while (byte != 0u) {
        if ((byte & 0xC0u) == 0xC0u) {
            if (lim - base < pos + 2u) return FB_DNS_UNEXPECTED_EOF;
            const uint32_t off = be16at(m, base + pos) & 0x3FFFu;
            if (off >= len) return FB_DNS_UNEXPECTED_EOF;
            if (ret < 0) ret = (int32_t)pos;
            if (off >= largest) return FB_DNS_BAD_POINTER;
            largest = off;
            pos = 0u;
            base = off;
            lim = len;
        } else if ((byte & 0xC0u) == 0u) {
            const uint32_t end = pos + byte + 1u;
            if (lim - base < end) return FB_DNS_UNEXPECTED_EOF;
            if (!m.ascii(base + pos + 1u, base + end)) return FB_DNS_LABEL_NOT_ASCII;
            pos = end;
            if (lim - base <= pos) return FB_DNS_UNEXPECTED_EOF;
        } else {
            return FB_DNS_UNKNOWN_LABEL_FORMAT;
        }
        byte = m(base + pos);
    }
    *blen = ret >= 0 ? (uint32_t)ret + 2u : pos + 1u;
    return FB_DNS_OK;
}

// Name's Display (labels joined by '.'; a pointer met after a label writes the '.' first) of a
// name that dns_name_scan accepted.  Writes at most cap - 1 bytes, four at a time (out is 4-byte
// aligned, bytes of the last dword past the name are zero); returns the full length and whether
// it ends with ".in-addr.arpa" / ".ip6.arpa", checked on a 16-byte window of the last bytes kept
// as four words (w0 byte 0 = the last byte), shifted by funnel shifts.
__device__ __forceinline__ bool window_ends(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t n,
                                            const char* sfx, uint32_t l) {
    if (n < l) return false;
    uint32_t e[4] = {0u, 0u, 0u, 0u}, m[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < l; ++k) {  // k-th byte from the end
        e[k >> 2] |= (uint32_t)(uint8_t)sfx[l - 1u - k] << (8u * (k & 3u));
        m[k >> 2] |= 0xFFu << (8u * (k & 3u));
    }
    return ((w0 ^ e[0]) & m[0]) == 0u && ((w1 ^ e[1]) & m[1]) == 0u && ((w2 ^ e[2]) & m[2]) == 0u &&
           ((w3 ^ e[3]) & m[3]) == 0u;
}

template <class M>
__device__ uint32_t dns_name_write(const M& m, uint32_t start, uint32_t* out, uint32_t cap, bool* reverse) {
    uint32_t seg = start, pos = start, n = 0u;
    uint32_t w0 = 0u, w1 = 0u, w2 = 0u, w3 = 0u, pend = 0u;
    auto put = [&](uint32_t c) {
        w3 = __builtin_amdgcn_alignbit(w3, w2, 24u);
        w2 = __builtin_amdgcn_alignbit(w2, w1, 24u);
        w1 = __builtin_amdgcn_alignbit(w1, w0, 24u);
        w0 = (w0 << 8) | c;
        if (n < cap - 1u) {
            pend |= c << (8u * (n & 3u));
            if ((n & 3u) == 3u) {
                out[n >> 2] = pend;
                pend = 0u;
            }
        }
        ++n;
    };
    for (;;) {
        const uint32_t b = m(pos);
        if (b == 0u) break;
        if ((b & 0xC0u) == 0xC0u) {
            if (pos != seg) put('.');
            pos = be16at(m, pos) & 0x3FFFu;
            seg = pos;
            continue;
        }
        if (pos != seg) put('.');
        for (uint32_t k = 1u; k <= b; ++k) put(m(pos + k));
        pos += b + 1u;
    }
    const uint32_t nw = min(n, cap - 1u);
    if (nw & 3u) out[nw >> 2] = pend;
    *reverse = window_ends(w0, w1, w2, w3, n, ".in-addr.arpa", 13u) || window_ends(w0, w1, w2, w3, n, ".ip6.arpa", 9u);
    return n;
}

__device__ __forceinline__ bool dns_qtype_ok(uint32_t t) {
    return (t >= 1u && t <= 16u && t != 3u) || t == 28u || t == 33u || (t >= 252u && t <= 255u);
}
__device__ __forceinline__ bool dns_type_ok(uint32_t t) {
    return (t >= 1u && t <= 16u && t != 3u) || t == 28u || t == 33u || t == 41u || t == 47u;
}

// One resource record at *off (parse_record); A / AAAA of the answer section are collected.
template <class M>
__device__ uint32_t dns_record(const M& m, uint32_t len, uint32_t* off, bool answer, fb_ip* addrs,
                               uint32_t* n_addrs, uint32_t* flags) {
    uint32_t bl;
    uint32_t st = dns_name_scan(m, len, *off, len, &bl);
    if (st) return st;
    uint32_t o = *off + bl;
    if (o + 10u > len) return FB_DNS_UNEXPECTED_EOF;
    const uint32_t typ = be16at(m, o);
    if (!dns_type_ok(typ)) return FB_DNS_INVALID_TYPE;
    const uint32_t cls = be16at(m, o + 2u) & 0x7FFFu;
    if (typ != 41u && !(cls >= 1u && cls <= 4u)) return FB_DNS_INVALID_CLASS;
    const uint32_t rdlen = be16at(m, o + 8u);
    o += 10u;
    if (o + rdlen > len) return FB_DNS_UNEXPECTED_EOF;
    const uint32_t end = o + rdlen;
    switch (typ) {
        case 1u:  // A
        case 28u: {  // AAAA
            const bool v6 = typ == 28u;
            if (rdlen != (v6 ? 16u : 4u)) return FB_DNS_WRONG_RDATA_LENGTH;
            if (answer) {
                if (*n_addrs < FB_DNS_MAX_ADDRS) {
                    fb_ip& a = addrs[*n_addrs];
                    a.family = v6 ? 10u : 2u;
                    a.reserved[0] = a.reserved[1] = a.reserved[2] = 0u;
                    for (int k = 0; k < 4; ++k)
                        a.addr[k] = (v6 || k == 0) ? (m(o + 4 * k) << 24 | m(o + 4 * k + 1) << 16 |
                                                      m(o + 4 * k + 2) << 8 | m(o + 4 * k + 3))
                                                   : 0u;
                    ++*n_addrs;
                } else {
                    *flags |= FB_DNS_ADDRS_TRUNCATED;
                }
            }
            break;
        }
        case 2u:
        case 5u:
        case 12u:  // NS CNAME PTR
            st = dns_name_scan(m, len, o, end, &bl);
            break;
        case 15u:  // MX
            if (rdlen < 3u) return FB_DNS_WRONG_RDATA_LENGTH;
            st = dns_name_scan(m, len, o + 2u, end, &bl);
            break;
        case 33u:  // SRV
            if (rdlen < 7u) return FB_DNS_WRONG_RDATA_LENGTH;
            st = dns_name_scan(m, len, o + 6u, end, &bl);
            break;
        case 6u: {  // SOA
            uint32_t b2;
            st = dns_name_scan(m, len, o, end, &bl);
            if (!st) st = dns_name_scan(m, len, o + bl, end, &b2);
            if (!st && end - (o + bl + b2) < 20u) st = FB_DNS_WRONG_RDATA_LENGTH;
            break;
        }
        case 16u: {  // TXT
            if (rdlen < 1u) return FB_DNS_WRONG_RDATA_LENGTH;
            uint32_t p = 0u;
            while (p < rdlen) {
                const uint32_t l = m(o + p);
                p += 1u;
                if (rdlen < l + p) return FB_DNS_WRONG_RDATA_LENGTH;
                p += l;
            }
            break;
        }
        default:
            break;
    }
    if (st) return st;
    *off = end;
    return FB_DNS_OK;
}

// Packet::parse of one message and the fields the resolver keeps (first question's name, A / AAAA
// answers); the record's *out.
template <class M>
__device__ void dns_message(const M& m, uint32_t len, uint32_t pkt_index, fb_ip* A, uint32_t* nm, fb_dns_msg* out) {
    fb_dns_msg r;
    r.pkt_index = pkt_index;
    r.id = 0;
    r.flags = 0;
    r.questions = r.answers = 0;
    r.name_len = 0;
    r.n_addrs = 0;
    r.reserved = 0;
    uint32_t st = FB_DNS_OK, flags = 0u, na = 0u;
    if (len < 12u) {
        st = FB_DNS_HEADER_TOO_SHORT;
    } else {
        r.id = (uint16_t)be16at(m, 0u);
        const uint32_t qd = be16at(m, 4u), an = be16at(m, 6u), ns = be16at(m, 8u), ar = be16at(m, 10u);
        r.questions = (uint16_t)qd;
        r.answers = (uint16_t)an;
        if ((m(2u) & 0x80u) == 0u) flags |= FB_DNS_QUERY;
        uint32_t off = 12u, q0 = 0u;
        for (uint32_t q = 0; q < qd && !st; ++q) {
            uint32_t bl;
            st = dns_name_scan(m, len, off, len, &bl);
            if (st) break;
            if (q == 0u) q0 = off;
            off += bl;
            if (off + 4u > len) { st = FB_DNS_UNEXPECTED_EOF; break; }
            if (!dns_qtype_ok(be16at(m, off))) { st = FB_DNS_INVALID_QUERY_TYPE; break; }
            const uint32_t qc = be16at(m, off + 2u) & 0x7FFFu;
            if (!((qc >= 1u && qc <= 4u) || qc == 255u)) { st = FB_DNS_INVALID_QUERY_CLASS; break; }
            off += 4u;
        }
        for (uint32_t k = 0; k < an + ns && !st; ++k) st = dns_record(m, len, &off, k < an, A, &na, &flags);
        bool opt = false;
        for (uint32_t k = 0; k < ar && !st; ++k) {
            if (off + 3u <= len && m(off) == 0u && m(off + 1u) == 0u && m(off + 2u) == 41u) {
                off += 1u;  // the OPT record's root name
                if (opt) { st = FB_DNS_ADDITIONAL_OPT; break; }
                opt = true;
                if (off + 10u > len) { st = FB_DNS_UNEXPECTED_EOF; break; }
                const uint32_t rdlen = be16at(m, off + 8u);
                off += 10u;
                if (off + rdlen > len) { st = FB_DNS_UNEXPECTED_EOF; break; }
                off += rdlen;
            } else {
                st = dns_record(m, len, &off, false, A, &na, &flags);
            }
        }
        if (!st && qd > 0u) {
            bool rev = false;
            const uint32_t nl = dns_name_write(m, q0, nm, FB_DNS_MAX_NAME, &rev);
            flags |= FB_DNS_HAS_QUESTION | (rev ? FB_DNS_REVERSE : 0u) | (nl > FB_DNS_MAX_NAME - 1u ? FB_DNS_NAME_TRUNCATED : 0u);
            r.name_len = (uint16_t)min(nl, FB_DNS_MAX_NAME - 1u);
        }
    }
    r.status = (uint8_t)st;
    r.flags = (uint8_t)(st ? 0u : flags);
    r.n_addrs = (uint8_t)(st ? 0u : na);
    *out = r;
}

// One wavefront (workgroup) per 64 messages.  The messages are first copied into LDS, one message
// per step of the wave with coalesced dword loads (range-checked buffer loads, so nothing is read
// past the frame buffer; only the dwords the message covers), up to kStage bytes each; each lane
// then parses its own message from LDS (17 KiB per wavefront: 9 per CU).
constexpr uint32_t kStage = 256;  // staged bytes per message (longer ones continue from HBM)
__global__ __launch_bounds__(64) void k_dns_parse(const uint8_t* frames, unsigned long long frames_bytes,
                                                  const fb_dns_out* dns, uint32_t n, const fb_batch_stats* stats,
                                                  fb_dns_msg* msgs, char* names, fb_ip* addrs) {
    __shared__ uint32_t s_msg[64][kStage / 4 + 1];  // +1 dword of row padding (lanes read different rows)
    const uint32_t lane = threadIdx.x;
    const uint32_t i0 = blockIdx.x * 64u, i = i0 + lane;
    const uint32_t cnt = stats ? (uint32_t)min((unsigned long long)n, stats->n_dns) : n;
    if (i0 >= cnt) return;  // uniform
    const bool live = i < cnt;
    const fb_dns_out d = dns[live ? i : i0];
    const unsigned long long lim = (unsigned long long)d.payload_offset + d.payload_length;
    const uint32_t len = (live && lim <= frames_bytes) ? d.payload_length : 0u;
    const uint32_t fb = (uint32_t)min(frames_bytes, (unsigned long long)0xFFFFFFFFull);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc((void*)frames, (short)0, (int)fb, 0x00020000);
    const uint32_t base = d.payload_offset & ~3u;
    // copy message j's dwords [base_j, base_j + kStage) with the whole wave (lane = dword), 32
    // messages' loads in flight before their LDS writes (a load-then-write per message would wait
    // out one HBM round trip per message); dwords past the message read as 0 (out-of-range offset)
    for (uint32_t j0 = 0; j0 < 64u; j0 += 32u) {
        uint32_t v[32];
#pragma unroll
        for (uint32_t u = 0; u < 32u; ++u) {
            const uint32_t bj = __builtin_amdgcn_readlane(base, (int)(j0 + u)), lj = __builtin_amdgcn_readlane(len, (int)(j0 + u));
            v[u] = __builtin_amdgcn_raw_buffer_load_b32(rf, 4u * lane < lj + 4u ? bj + 4u * lane : 0xFFFFFFF0u, 0, 0);
        }
#pragma unroll
        for (uint32_t u = 0; u < 32u; ++u) s_msg[j0 + u][lane] = v[u];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!live) return;
    const uint32_t mis = d.payload_offset & 3u;
    fb_ip* A = addrs + (size_t)i * FB_DNS_MAX_ADDRS;
    uint32_t* nm = reinterpret_cast<uint32_t*>(names + (size_t)i * FB_DNS_MAX_NAME);  // 4-B aligned (fb_dns_parse_dev)
    // the copy starts at the dword holding the first byte: kStage - mis message bytes are staged;
    // when every live lane's message is whole in LDS the wave runs the LDS-only parse (no
    // per-byte range branch, dword-wide label checks)
    if (__all(len <= kStage - mis)) {
        dns_message(MsgLds{s_msg[lane], mis}, len, d.pkt_index, A, nm, msgs + i);
    } else {
        dns_message(MsgMixed{reinterpret_cast<const uint8_t*>(s_msg[lane]) + mis, rf, d.payload_offset, kStage - mis},
                    len, d.pkt_index, A, nm, msgs + i);
    }
}

hipError_t launch_dns_parse(const uint8_t* frames, unsigned long long frames_bytes, const fb_dns_out* dns, uint32_t n,
                            const fb_batch_stats* stats, fb_dns_msg* msgs, char* names, fb_ip* addrs, hipStream_t s) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(k_dns_parse, dim3((n + 63u) / 64u), dim3(64), 0, s, frames, frames_bytes, dns, n, stats, msgs,
                       names, addrs);
    return hipGetLastError();
}

}  // namespace fbk
