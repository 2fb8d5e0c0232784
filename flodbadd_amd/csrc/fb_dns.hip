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

__device__ __forceinline__ uint32_t be16at(const uint8_t* m, uint32_t i) { return ((uint32_t)m[i] << 8) | m[i + 1]; }

// Name::scan over the slice m[start..limit) with pointers into m[0..len); *blen = byte_len().
__device__ uint32_t dns_name_scan(const uint8_t* m, uint32_t len, uint32_t start, uint32_t limit, uint32_t* blen) {
    uint32_t base = start, lim = limit, pos = 0u;
    if (lim <= base) return FB_DNS_UNEXPECTED_EOF;
    uint32_t largest = len;
    int32_t ret = -1;
    uint32_t byte = m[base];
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
            for (uint32_t k = pos + 1u; k < end; ++k)
                if (m[base + k] >= 0x80u) return FB_DNS_LABEL_NOT_ASCII;
            pos = end;
            if (lim - base <= pos) return FB_DNS_UNEXPECTED_EOF;
        } else {
            return FB_DNS_UNKNOWN_LABEL_FORMAT;
        }
        byte = m[base + pos];
    }
    *blen = ret >= 0 ? (uint32_t)ret + 2u : pos + 1u;
    return FB_DNS_OK;
}

// Name's Display (labels joined by '.'; a pointer met after a label writes the '.' first) of a
// name that dns_name_scan accepted.  Writes at most cap - 1 bytes; returns the full length and
// whether it ends with ".in-addr.arpa" / ".ip6.arpa" (checked on a 16-byte tail window).
__device__ uint32_t dns_name_write(const uint8_t* m, uint32_t start, char* out, uint32_t cap, bool* reverse) {
    uint32_t seg = start, pos = start, n = 0u;
    uint8_t tail[16];
    for (int k = 0; k < 16; ++k) tail[k] = 0;
    auto put = [&](uint8_t c) {
        if (n < cap - 1u) out[n] = (char)c;
        tail[n & 15u] = c;
        ++n;
    };
    for (;;) {
        const uint32_t b = m[pos];
        if (b == 0u) break;
        if ((b & 0xC0u) == 0xC0u) {
            if (pos != seg) put('.');
            pos = be16at(m, pos) & 0x3FFFu;
            seg = pos;
            continue;
        }
        if (pos != seg) put('.');
        for (uint32_t k = 1u; k <= b; ++k) put(m[pos + k]);
        pos += b + 1u;
    }
    auto ends = [&](const char* sfx, uint32_t l) {
        if (n < l) return false;
        for (uint32_t k = 0; k < l; ++k)
            if (tail[(n - l + k) & 15u] != (uint8_t)sfx[k]) return false;
        return true;
    };
    *reverse = ends(".in-addr.arpa", 13u) || ends(".ip6.arpa", 9u);
    return n;
}

__device__ __forceinline__ bool dns_qtype_ok(uint32_t t) {
    return (t >= 1u && t <= 16u && t != 3u) || t == 28u || t == 33u || (t >= 252u && t <= 255u);
}
__device__ __forceinline__ bool dns_type_ok(uint32_t t) {
    return (t >= 1u && t <= 16u && t != 3u) || t == 28u || t == 33u || t == 41u || t == 47u;
}

// One resource record at *off (parse_record); A / AAAA of the answer section are collected.
__device__ uint32_t dns_record(const uint8_t* m, uint32_t len, uint32_t* off, bool answer, fb_ip* addrs,
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
                        a.addr[k] = (v6 || k == 0) ? ((uint32_t)m[o + 4 * k] << 24 | (uint32_t)m[o + 4 * k + 1] << 16 |
                                                      (uint32_t)m[o + 4 * k + 2] << 8 | m[o + 4 * k + 3])
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
                const uint32_t l = m[o + p];
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

__global__ __launch_bounds__(64) void k_dns_parse(const uint8_t* frames, unsigned long long frames_bytes,
                                                  const fb_dns_out* dns, uint32_t n, const fb_batch_stats* stats,
                                                  fb_dns_msg* msgs, char* names, fb_ip* addrs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cnt = stats ? (uint32_t)min((unsigned long long)n, stats->n_dns) : n;
    if (i >= cnt) return;
    const fb_dns_out d = dns[i];
    fb_dns_msg r;
    r.pkt_index = d.pkt_index;
    r.id = 0;
    r.flags = 0;
    r.questions = r.answers = 0;
    r.name_len = 0;
    r.n_addrs = 0;
    r.reserved = 0;
    uint32_t st = FB_DNS_OK, flags = 0u, na = 0u;
    const unsigned long long lim = (unsigned long long)d.payload_offset + d.payload_length;
    const uint32_t len = lim <= frames_bytes ? d.payload_length : 0u;
    const uint8_t* m = frames + d.payload_offset;
    fb_ip* A = addrs + (size_t)i * FB_DNS_MAX_ADDRS;
    char* name = names + (size_t)i * FB_DNS_MAX_NAME;
    if (len < 12u) {
        st = FB_DNS_HEADER_TOO_SHORT;
    } else {
        r.id = (uint16_t)be16at(m, 0u);
        const uint32_t qd = be16at(m, 4u), an = be16at(m, 6u), ns = be16at(m, 8u), ar = be16at(m, 10u);
        r.questions = (uint16_t)qd;
        r.answers = (uint16_t)an;
        if ((m[2] & 0x80u) == 0u) flags |= FB_DNS_QUERY;
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
            if (off + 3u <= len && m[off] == 0u && m[off + 1u] == 0u && m[off + 2u] == 41u) {
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
            const uint32_t nl = dns_name_write(m, q0, name, FB_DNS_MAX_NAME, &rev);
            flags |= FB_DNS_HAS_QUESTION | (rev ? FB_DNS_REVERSE : 0u) | (nl > FB_DNS_MAX_NAME - 1u ? FB_DNS_NAME_TRUNCATED : 0u);
            r.name_len = (uint16_t)min(nl, FB_DNS_MAX_NAME - 1u);
        }
    }
    r.status = (uint8_t)st;
    r.flags = (uint8_t)(st ? 0u : flags);
    r.n_addrs = (uint8_t)(st ? 0u : na);
    msgs[i] = r;
}

hipError_t launch_dns_parse(const uint8_t* frames, unsigned long long frames_bytes, const fb_dns_out* dns, uint32_t n,
                            const fb_batch_stats* stats, fb_dns_msg* msgs, char* names, fb_ip* addrs, hipStream_t s) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(k_dns_parse, dim3((n + 63u) / 64u), dim3(64), 0, s, frames, frames_bytes, dns, n, stats, msgs,
                       names, addrs);
    return hipGetLastError();
}

}  // namespace fbk
