/*
 * oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (see oracle.h).  Plain C99, single-threaded, written for clarity rather than speed, but
 * without gratuitous overhead so it can also serve as the bench's cpu_baseline ("port").
 *
 * Every function cites the reference lines it restates.  Byte-level decode follows
 * pnet_packet 0.35.0 (Cargo.lock:2588), which is not vendored under /root/reference:
 * the rules below are the published crate's accessor/payload semantics as restated in
 * SURVEY.md §8a "a1 exact decode rules" -- parity of the decode step is UNPINNED by any
 * reference test (no reference test builds raw frames).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define TCP_FIN 0x01u
#define TCP_SYN 0x02u
#define TCP_RST 0x04u
#define TCP_PSH 0x08u
#define TCP_ACK 0x10u

static uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* ---------------------------------------------------------------------------------------
 * parse_packet_pcap, src/packets.rs:603-802.
 * EthernetPacket::new needs >= 14 bytes; payload() is the rest of the frame (pnet ethernet).
 * Ipv4Packet::new needs >= 20 bytes; payload() = packet[20+opt .. min(20+opt+plen, len)]
 *   with opt = sat(ihl*4 - 20), plen = sat(total_length - ihl*4), empty if len <= 20+opt.
 * Ipv6Packet::new needs >= 40 bytes; payload() = packet[40 .. min(40+payload_length, len)].
 * TcpPacket::new needs >= 20 bytes; payload() = packet[20+opt ..] (opt = doff>5 ? doff*4-20 : 0),
 *   empty if len <= 20+opt.  UdpPacket::new needs >= 8; payload() = packet[8..] (length
 *   field ignored).
 * ------------------------------------------------------------------------------------- */
static uint32_t parse_l4(const uint8_t* frame, uint32_t l4_off, uint32_t l4_len, uint32_t proto,
                         orc_parsed* o) {
    const uint8_t* P = frame + l4_off;
    if (proto == 6) { /* IpNextHeaderProtocols::Tcp, src/packets.rs:624-665 / 707-749 */
        if (l4_len < 20) return ORC_NONE;            /* "Failed to parse TCP packet" */
        uint32_t doff = P[12] >> 4;
        uint32_t hs = 20 + (doff > 5 ? doff * 4 - 20 : 0);
        uint32_t plen = l4_len <= hs ? 0 : l4_len - hs;
        o->protocol = 6;
        o->src_port = (uint16_t)be16(P);
        o->dst_port = (uint16_t)be16(P + 2);
        o->flags = P[13]; /* tcp.get_flags() is u8, src/packets.rs:635 */
        o->has_flags = 1;
        o->packet_length = plen;
        if (o->src_port == 53 || o->dst_port == 53) { /* DNS over TCP, src/packets.rs:638-650 */
            if (plen < 2) return ORC_NONE;           /* "DNS-over-TCP payload too short" */
            o->dns_payload_offset = l4_off + hs + 2; /* drain(0..2) */
            o->dns_payload_length = plen - 2;
            return ORC_DNS;
        }
        return ORC_SESSION;
    }
    if (proto == 17) { /* IpNextHeaderProtocols::Udp, src/packets.rs:667-699 / 750-783 */
        if (l4_len < 8) return ORC_NONE; /* "Failed to parse UDP packet" */
        o->protocol = 17;
        o->src_port = (uint16_t)be16(P);
        o->dst_port = (uint16_t)be16(P + 2);
        o->flags = 0;
        o->has_flags = 0; /* flags: None */
        o->packet_length = l4_len - 8;
        if (o->src_port == 53 || o->dst_port == 53) { /* DNS over UDP, src/packets.rs:681-686 */
            o->dns_payload_offset = l4_off + 8;
            o->dns_payload_length = l4_len - 8;
            return ORC_DNS;
        }
        return ORC_SESSION;
    }
    return ORC_NONE; /* `_ => None` */
}

uint32_t orc_parse_packet_pcap(const uint8_t* f, uint32_t L, orc_parsed* o) {
    memset(o, 0, sizeof(*o));
    if (L < 14) return ORC_NONE; /* "Failed to parse Ethernet packet", src/packets.rs:604-610 */
    uint32_t et = be16(f + 12);
    const uint8_t* ip = f + 14;
    uint32_t n = L - 14;
    uint32_t kind = ORC_NONE;
    if (et == 0x0800) { /* EtherTypes::Ipv4, src/packets.rs:612 */
        if (n < 20) return ORC_NONE;
        uint32_t ihl4 = (ip[0] & 15u) * 4u; /* version is not checked by pnet */
        uint32_t tot = be16(ip + 2);
        uint32_t start = 20 + (ihl4 > 20 ? ihl4 - 20 : 0);
        uint32_t plen = tot > ihl4 ? tot - ihl4 : 0;
        uint32_t l4_len = 0;
        if (n > start) {
            uint32_t end = start + plen < n ? start + plen : n;
            l4_len = end - start;
        }
        o->family = 2;
        o->src_ip[0] = be32(ip + 12); /* u32::from(Ipv4Addr), src/l7_ebpf.rs:85 */
        o->dst_ip[0] = be32(ip + 16);
        o->ip_packet_length = tot; /* get_total_length(), src/packets.rs:620 */
        kind = parse_l4(f, 14 + start, l4_len, ip[9], o);
    } else if (et == 0x86DD) { /* EtherTypes::Ipv6, src/packets.rs:701 */
        if (n < 40) return ORC_NONE;
        uint32_t plen6 = be16(ip + 4);
        uint32_t l4_len = 0;
        if (n > 40) {
            uint32_t end = 40 + plen6 < n ? 40 + plen6 : n;
            l4_len = end - 40;
        }
        o->family = 10;
        for (int k = 0; k < 4; ++k) {
            o->src_ip[k] = be32(ip + 8 + 4 * k);
            o->dst_ip[k] = be32(ip + 24 + 4 * k);
        }
        o->ip_packet_length = plen6 + 40; /* src/packets.rs:709 */
        kind = parse_l4(f, 14 + 40, l4_len, ip[6], o); /* next header, no ext-hdr walk */
    } else {
        return ORC_NONE; /* `_ => None`, src/packets.rs:800 (VLAN, ARP, ... included) */
    }
    o->kind = kind;
    return kind;
}

/* get_name_from_port(p) != "" (src/port_vulns.rs:213-228, src/packets.rs:233-237). */
int orc_is_service_port(const orc_cfg* c, uint16_t p) {
    return (c->service_bitmap[p >> 3] >> (p & 7)) & 1;
}

/* is_lan_ipv4_fast, src/ip.rs:55-91. */
static int is_lan_v4(uint32_t v) {
    if (v == 0 || v == 0xFFFFFFFFu) return 1;
    if ((v >> 24) == 127) return 1;
    if ((v >> 28) == 0xE) return 1;
    if ((v >> 16) == 0xA9FE) return 1;
    if ((v >> 24) == 10) return 1;
    if ((v >> 24) == 172) {
        uint32_t s = (v >> 16) & 0xFF;
        if (s >= 16 && s <= 31) return 1;
    }
    if ((v >> 16) == 0xC0A8) return 1;
    return 0;
}

/* is_local_ipv6 (src/ip.rs:112-134) then is_lan_ipv6_fast (src/ip.rs:139-156). */
static int is_lan_v6(const orc_cfg* c, const uint32_t w[4]) {
    uint32_t seg0 = w[0] >> 16;
    if ((w[0] | w[1] | w[2] | w[3]) == 0) return 1;                        /* :: */
    if (w[0] == 0 && w[1] == 0 && w[2] == 0 && w[3] == 1) return 1;        /* ::1 */
    if ((seg0 & 0xffc0u) == 0xfe80u) return 1;                             /* fe80::/10 */
    if ((seg0 & 0xff00u) == 0xff00u) return 1;                             /* ff00::/8 */
    if ((seg0 & 0xfe00u) == 0xfc00u) return 1;                             /* fc00::/7 */
    for (uint32_t i = 0; i < c->n_lan_v6; ++i) {
        uint32_t pfx = c->lan_v6[i].prefix;
        int match = 1;
        for (int k = 0; k < 4; ++k) {
            /* mask = !0u128 << (128 - prefix) (prefix 0 -> 0), src/ip.rs:143-147 */
            int bits = (int)pfx - 32 * k;
            uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : 0xFFFFFFFFu << (32 - bits));
            if ((w[k] & m) != c->lan_v6[i].net[k]) { match = 0; break; }
        }
        if (match) return 1;
    }
    return 0;
}

/* is_lan_ip, src/ip.rs:199-242 (the known-local cache only memoises true results). */
int orc_is_lan_ip(const orc_cfg* c, uint32_t family, const uint32_t ip[4]) {
    return family == 2 ? is_lan_v4(ip[0]) : is_lan_v6(c, ip);
}

static int is_own_ip(const orc_cfg* c, uint32_t family, const uint32_t ip[4]) {
    for (uint32_t i = 0; i < c->n_own_ips; ++i) {
        const fb_ip* o = &c->own_ips[i];
        if (o->family != family) continue;
        if (family == 2 ? o->addr[0] == ip[0]
                        : (o->addr[0] == ip[0] && o->addr[1] == ip[1] && o->addr[2] == ip[2] &&
                           o->addr[3] == ip[3]))
            return 1;
    }
    return 0;
}

/* map_tcp_flags, src/packets.rs:561-601. */
char orc_map_tcp_flags(uint8_t fl, uint32_t plen, int orig) {
    if ((fl & TCP_SYN) && !(fl & TCP_ACK)) return orig ? 'S' : 's';
    if ((fl & TCP_SYN) && (fl & TCP_ACK)) return orig ? 'H' : 'h';
    if (fl & TCP_FIN) return orig ? 'F' : 'f';
    if (fl & TCP_RST) return orig ? 'R' : 'r';
    if (plen > 0) return orig ? '>' : '<';
    if (fl & TCP_ACK) return orig ? 'A' : 'a';
    return '-';
}

/* Key canonicalisation + originator + filter: src/packets.rs:232-327. */
uint32_t orc_classify(const orc_cfg* c, const orc_parsed* p, uint32_t pkt_index, fb_pkt_out* r) {
    int S = orc_is_service_port(c, p->src_port);
    int D = orc_is_service_port(c, p->dst_port);
    int swap;
    if (S && !D) {
        swap = 1; /* source is likely a server (src/packets.rs:245-253) */
    } else if (S && D) {
        if (p->has_flags) {
            if (p->protocol == 6 && (p->flags & TCP_SYN) && !(p->flags & TCP_ACK))
                swap = 0; /* SYN without ACK (src/packets.rs:257-263) */
            else if (p->protocol == 6 && (p->flags & TCP_SYN) && (p->flags & TCP_ACK))
                swap = 1; /* SYN+ACK (src/packets.rs:264-275) */
            else
                swap = p->src_port < p->dst_port; /* port tiebreak (src/packets.rs:276-292) */
        } else {
            swap = p->src_port < p->dst_port; /* UDP tiebreak (src/packets.rs:294-307) */
        }
    } else {
        swap = 0;
    }
    memset(r, 0, sizeof(*r));
    const uint32_t* ks = swap ? p->dst_ip : p->src_ip;
    const uint32_t* kd = swap ? p->src_ip : p->dst_ip;
    for (int k = 0; k < 4; ++k) {
        r->key.src_ip[k] = ks[k];
        r->key.dst_ip[k] = kd[k];
    }
    r->key.src_port = swap ? p->dst_port : p->src_port;
    r->key.dst_port = swap ? p->src_port : p->dst_port;
    r->key.protocol = p->protocol;
    r->key.family = p->family;
    r->packet_length = p->packet_length;
    r->ip_packet_length = p->ip_packet_length;
    r->tcp_flags = p->has_flags ? p->flags : 0;
    r->pkt_index = pkt_index;

    /* is_originator, src/packets.rs:316-319: field-wise equality raw vs key. */
    int orig = memcmp(p->src_ip, r->key.src_ip, 16) == 0 && p->src_port == r->key.src_port &&
               memcmp(p->dst_ip, r->key.dst_ip, 16) == 0 && p->dst_port == r->key.dst_port;

    uint8_t meta = 0;
    if (p->has_flags) meta |= FB_META_HAS_FLAGS;
    if (swap) meta |= FB_META_SWAP;
    if (orig) meta |= FB_META_ORIGINATOR;
    int lan_ks = orc_is_lan_ip(c, p->family, r->key.src_ip);
    int lan_kd = orc_is_lan_ip(c, p->family, r->key.dst_ip);
    if (lan_ks) meta |= FB_META_LOCAL_SRC;
    if (lan_kd) meta |= FB_META_LOCAL_DST;
    if (is_own_ip(c, p->family, r->key.src_ip)) meta |= FB_META_SELF_SRC;
    if (is_own_ip(c, p->family, r->key.dst_ip)) meta |= FB_META_SELF_DST;
    /* dst_service: name of key.dst_port (src/packets.rs:441-464) */
    if (orc_is_service_port(c, r->key.dst_port)) meta |= FB_META_DST_SERVICE;
    r->meta = meta;
    r->hist_char = p->has_flags ? (uint8_t)orc_map_tcp_flags(p->flags, p->packet_length, orig) : 0;

    /* Filter (src/packets.rs:321-327) on the raw packet's session; is_local_session! =
     * is_lan(src) && is_lan(dst) (src/sessions.rs:660-672) -- symmetric, so key order is moot. */
    int local = lan_ks && lan_kd;
    if (c->filter == FB_FILTER_LOCAL_ONLY && !local) return FB_CLASS_FILTERED;
    if (c->filter == FB_FILTER_GLOBAL_ONLY && local) return FB_CLASS_FILTERED;
    return FB_CLASS_SESSION;
}

int orc_parse_classify(const orc_cfg* c, const uint8_t* frames, uint64_t frames_bytes,
                       const uint32_t* offsets, uint32_t n, fb_pkt_out* out, uint32_t* n_out,
                       fb_dns_out* dns, uint32_t* n_dns, uint8_t* cls, fb_batch_stats* st) {
    fb_batch_stats s;
    memset(&s, 0, sizeof(s));
    uint32_t no = 0, nd = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t o0 = offsets[i], o1 = offsets[i + 1];
        uint32_t k;
        orc_parsed p;
        if (o1 < o0 || (uint64_t)o1 > frames_bytes) {
            s.bad_offsets++;
            k = FB_CLASS_DROP;
        } else {
            uint32_t kind = orc_parse_packet_pcap(frames + o0, o1 - o0, &p);
            if (kind == ORC_NONE) {
                k = FB_CLASS_DROP;
            } else if (kind == ORC_DNS) {
                k = FB_CLASS_DNS;
                if (dns) {
                    fb_dns_out* d = &dns[nd];
                    d->pkt_index = i;
                    d->payload_offset = o0 + p.dns_payload_offset;
                    d->payload_length = p.dns_payload_length;
                    d->protocol = p.protocol;
                    d->family = p.family;
                    d->reserved = 0;
                }
                nd++;
            } else {
                /* PACKET_STATS increments precede the filter (src/packets.rs:211-227). */
                s.total_processed++;
                if (p.protocol == 6) s.tcp_processed++; else s.udp_processed++;
                if (p.family == 2) s.ipv4_processed++; else s.ipv6_processed++;
                fb_pkt_out rec;
                k = orc_classify(c, &p, i, &rec);
                if (k == FB_CLASS_SESSION) {
                    if (out) out[no] = rec;
                    no++;
                }
            }
        }
        if (k == FB_CLASS_DROP) s.n_drop++;
        if (k == FB_CLASS_FILTERED) s.n_filtered++;
        if (cls) cls[i] = (uint8_t)k;
    }
    s.n_session = no;
    s.n_dns = nd;
    if (n_out) *n_out = no;
    if (n_dns) *n_dns = nd;
    if (st) *st = s;
    return 0;
}

int orc_process_parsed(const orc_cfg* c, const fb_parsed_pkt* in, uint32_t n, fb_pkt_out* out,
                       uint32_t* n_out, uint8_t* cls, fb_batch_stats* st) {
    fb_batch_stats s;
    memset(&s, 0, sizeof(s));
    uint32_t no = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const fb_parsed_pkt* q = &in[i];
        uint32_t k = FB_CLASS_DROP;
        if ((q->session.protocol == 6 || q->session.protocol == 17) &&
            (q->session.family == 2 || q->session.family == 10)) {
            orc_parsed p;
            memset(&p, 0, sizeof(p));
            p.kind = ORC_SESSION;
            p.protocol = q->session.protocol;
            p.family = q->session.family;
            p.has_flags = q->has_flags ? 1 : 0;
            p.flags = q->tcp_flags;
            memcpy(p.src_ip, q->session.src_ip, 16);
            memcpy(p.dst_ip, q->session.dst_ip, 16);
            p.src_port = q->session.src_port;
            p.dst_port = q->session.dst_port;
            p.packet_length = q->packet_length;
            p.ip_packet_length = q->ip_packet_length;
            s.total_processed++; /* PACKET_STATS, src/packets.rs:211-227 */
            if (p.protocol == 6) s.tcp_processed++; else s.udp_processed++;
            if (p.family == 2) s.ipv4_processed++; else s.ipv6_processed++;
            fb_pkt_out rec;
            k = orc_classify(c, &p, q->pkt_index, &rec);
            if (k == FB_CLASS_SESSION) {
                if (out) out[no] = rec;
                no++;
            }
        }
        if (k == FB_CLASS_DROP) s.n_drop++;
        if (k == FB_CLASS_FILTERED) s.n_filtered++;
        if (cls) cls[i] = (uint8_t)k;
    }
    s.n_session = no;
    if (n_out) *n_out = no;
    if (st) *st = s;
    return 0;
}

/* ---------------------------------------------------------------------------------------
 * Session table: a restatement of the DashMap<Session, SessionInfo> upsert
 * (src/packets.rs:329-535) keeping the integer counters (src/packets.rs:111-120, 383-391),
 * the history string and conn_state (src/packets.rs:187-198, 410-426, 539-559).
 * Open addressing with FNV-1a over the 40-byte key (the reference hashes with SipHash and a
 * random key, so no hash value is a parity target -- only keys and counters are).
 * ------------------------------------------------------------------------------------- */
typedef struct orc_flow {
    fb_flow_rec rec;
    char* hist;
    uint64_t hist_len, hist_cap;
    char conn_state[4];
    int ended; /* end_time.is_some() */
    int used;
    uint32_t char_call[4]; /* update call of the first S, s, H, h (FB_CALL_NONE: none), for the merge */
    fb_flow_time tm;       /* timed contexts: capture-time state (packets.rs:137-186, 352-426) */
    double ref_total_s;    /* the reference's own f64 running sum total_segment_interarrival */
    double ref_ia_s;       /* and its segment_interarrival */
} orc_flow;

struct orc_flows {
    orc_flow* slots;
    uint64_t cap, count;
    uint32_t batch; /* update calls since new/clear: the high word of fb_flow_rec positions */
};

static uint64_t key_hash(const fb_session_key* k) {
    const uint8_t* b = (const uint8_t*)k;
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 40; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h;
}

orc_flows* orc_flows_new(void) {
    orc_flows* f = (orc_flows*)calloc(1, sizeof(orc_flows));
    f->cap = 1024;
    f->slots = (orc_flow*)calloc(f->cap, sizeof(orc_flow));
    return f;
}

void orc_flows_clear(orc_flows* f) {
    for (uint64_t i = 0; i < f->cap; ++i) free(f->slots[i].hist);
    memset(f->slots, 0, f->cap * sizeof(orc_flow));
    f->count = 0;
    f->batch = 0;
}

void orc_flows_free(orc_flows* f) {
    if (!f) return;
    for (uint64_t i = 0; i < f->cap; ++i) free(f->slots[i].hist);
    free(f->slots);
    free(f);
}

static orc_flow* find_slot(orc_flow* slots, uint64_t cap, const fb_session_key* k) {
    uint64_t i = key_hash(k) & (cap - 1);
    for (;;) {
        if (!slots[i].used || memcmp(&slots[i].rec.key, k, sizeof(*k)) == 0) return &slots[i];
        i = (i + 1) & (cap - 1);
    }
}

static void grow(orc_flows* f) {
    uint64_t ncap = f->cap * 2;
    orc_flow* ns = (orc_flow*)calloc(ncap, sizeof(orc_flow));
    for (uint64_t i = 0; i < f->cap; ++i)
        if (f->slots[i].used) *find_slot(ns, ncap, &f->slots[i].rec.key) = f->slots[i];
    free(f->slots);
    f->slots = ns;
    f->cap = ncap;
}

/* determine_conn_state, src/packets.rs:539-559: scans the history string as the reference does.
 * Returns the fb_conn_state code and writes the string. */
static uint8_t conn_state_of(const char* h, uint64_t n, char out[4]) {
    int has[128] = {0};
    for (uint64_t i = 0; i < n; ++i) has[(unsigned char)h[i] & 127] = 1;
    const char* s;
    uint8_t code;
    if (has['S'] && has['H'] && has['F'] && has['f']) { s = "SF"; code = FB_CONN_SF; }
    else if (has['S'] && !has['h'] && !has['r']) { s = "S0"; code = FB_CONN_S0; }
    else if (has['R'] || has['r']) { s = "REJ"; code = FB_CONN_REJ; }
    else if (has['S'] && has['H'] && !has['F'] && !has['f']) { s = "S1"; code = FB_CONN_S1; }
    else { s = "-"; code = FB_CONN_OTHER; }
    strcpy(out, s);
    return code;
}

/* Position of FB_HIST_CHARS holding c (16 when absent). */
static uint32_t hist_bit(char c) {
    const char* p = strchr(FB_HIST_CHARS, c);
    return (c && p) ? (uint32_t)(p - FB_HIST_CHARS) : 16u;
}

static void flow_upsert(orc_flows* f, const fb_pkt_out* r, fb_batch_stats* st, const uint64_t* ts);

void orc_flows_update(orc_flows* f, const fb_pkt_out* recs, uint64_t n, fb_batch_stats* st) {
    for (uint64_t i = 0; i < n; ++i) flow_upsert(f, &recs[i], st, NULL);
    f->batch++;
}

void orc_flows_update_timed(orc_flows* f, const fb_pkt_out* recs, uint64_t n, fb_batch_stats* st,
                            const uint64_t* ts) {
    for (uint64_t i = 0; i < n; ++i) flow_upsert(f, &recs[i], st, ts);
    f->batch++;
}

/* (now - then).num_milliseconds(): chrono's TimeDelta between two instants, truncated toward zero
 * (timestamps are ns since an epoch, as i64 -- DateTime<Utc>'s range) */
static int64_t ms_between(uint64_t now, uint64_t then) { return ((int64_t)now - (int64_t)then) / 1000000; }

/* The segment state of update_session_stats (src/packets.rs:137-186) at capture time `now`. */
static void segment_update(orc_flow* s, int tcp_psh, uint64_t now) {
    fb_flow_time* t = &s->tm;
    const double since_s = (double)ms_between(now, t->last_activity_ns) / 1000.0; /* 138 */
    const int timeout = since_s >= 5.0;                                              /* segment_timeout */
    const int is_end = tcp_psh || (t->in_segment && timeout);                       /* 140-149 */
    if (!t->in_segment) {                                                            /* 151-154 */
        t->in_segment = 1;
        t->current_segment_start_ns = now;
    }
    if (is_end && t->in_segment) {                                                   /* 156-186 */
        const uint64_t prev = t->last_segment_end_ns;
        t->segment_count += 1;
        t->in_segment = 0;
        t->last_segment_end_ns = now;
        if (prev != FB_SEEN_NONE) {
            const int64_t ia_ms = ms_between(t->current_segment_start_ns, prev);
            const double seg_ia = (double)ia_ms / 1000.0;
            if (seg_ia >= 0.0) {
                t->total_segment_interarrival_ms += ia_ms;
                s->ref_total_s += seg_ia;
                s->ref_ia_s = t->segment_count > 1 ? s->ref_total_s / (double)(t->segment_count - 1) : 0.0;
                t->segment_interarrival_div = t->segment_count > 1 ? t->segment_count - 1 : 0;
            } /* else: warn! and skip (src/packets.rs:172-179) */
        }
        if (timeout) {
            t->in_segment = 1;
            t->current_segment_start_ns = now;
        }
    }
    t->last_activity_ns = now; /* 189 */
}

/* One SessionPacketData through the DashMap upsert (src/packets.rs:329-535); `ts` (timed): the
 * batch's per-frame capture timestamps, ts[pkt_index] = the packet's `now`. */
static void flow_upsert(orc_flows* f, const fb_pkt_out* r, fb_batch_stats* st, const uint64_t* ts) {
    {
        if ((f->count + 1) * 2 > f->cap) grow(f);
        orc_flow* s = find_slot(f->slots, f->cap, &r->key);
        const uint64_t pos = ((uint64_t)f->batch << 32) | r->pkt_index; /* stands for `now` */
        const int tcp_psh = (r->meta & FB_META_HAS_FLAGS) && r->key.protocol == 6 && (r->tcp_flags & TCP_PSH);
        const int inserted = !s->used;
        if (!s->used) { /* Entry::Vacant, src/packets.rs:344 */
            memset(s, 0, sizeof(*s));
            s->used = 1;
            s->rec.key = r->key;
            s->rec.first_seen = pos; /* start_time, src/packets.rs:352 */
            s->rec.end_seen = FB_SEEN_NONE;
            /* is_local_src/dst, is_self_src/dst of the key (src/packets.rs:429-435) and dst_service
               (src/packets.rs:441-466), stored once at insert */
            s->rec.session_flags = ((uint32_t)r->meta >> 3) & 0x1Fu;
            for (int b = 0; b < 4; ++b) s->char_call[b] = FB_CALL_NONE;
            f->count++;
            if (st) st->new_sessions++;
        } else if (st) {
            st->updated_sessions++; /* Entry::Occupied, src/packets.rs:332 */
        }
        if (r->meta & FB_META_ORIGINATOR) {
            s->rec.outbound_bytes += r->packet_length;
            s->rec.orig_pkts += 1;
            s->rec.orig_ip_bytes += r->ip_packet_length;
        } else {
            s->rec.inbound_bytes += r->packet_length;
            s->rec.resp_pkts += 1;
            s->rec.resp_ip_bytes += r->ip_packet_length;
        }
        if (!ts) {
            /* segment detection without the wall-clock timeout (src/packets.rs:137-160 update, 370-376
               and 414-420 insert): a TCP packet with PSH ends the segment -- segment_count += 1,
               in_segment = false --; any other packet leaves the flow in a segment (a new one starts
               when it was not) */
            if (tcp_psh) s->rec.segment_count += 1;
            s->rec.in_segment = tcp_psh ? 0 : 1;
        } else {
            const uint64_t now = ts[r->pkt_index];
            fb_flow_time* t = &s->tm;
            if (inserted) { /* SessionStats at insert (src/packets.rs:352-380, 414-420) */
                t->start_time_ns = t->last_activity_ns = t->current_segment_start_ns = now;
                t->end_time_ns = t->last_segment_end_ns = FB_SEEN_NONE;
                t->in_segment = 1;
                if (tcp_psh) {
                    t->segment_count = 1;
                    t->in_segment = 0;
                    t->last_segment_end_ns = now;
                }
            } else {
                segment_update(s, tcp_psh, now);
            }
            /* end_time at the first FIN/RST (src/packets.rs:195-198, 423-426) */
            if ((r->meta & FB_META_HAS_FLAGS) && (r->tcp_flags & (TCP_FIN | TCP_RST)) && t->end_time_ns == FB_SEEN_NONE)
                t->end_time_ns = now;
            s->rec.segment_count = t->segment_count;
            s->rec.in_segment = t->in_segment;
        }
        if (r->meta & FB_META_HAS_FLAGS) { /* history push, src/packets.rs:187-198, 410-426 */
            if (s->hist_len + 1 > s->hist_cap) {
                s->hist_cap = s->hist_cap ? s->hist_cap * 2 : 16;
                s->hist = (char*)realloc(s->hist, s->hist_cap);
            }
            s->hist[s->hist_len++] = (char)r->hist_char;
            s->rec.hist_len = (uint32_t)s->hist_len;
            const uint32_t b = hist_bit((char)r->hist_char);
            if (b < 16u) s->rec.hist_mask |= (uint16_t)(1u << b);
            if (b < 4u && s->char_call[b] == FB_CALL_NONE) s->char_call[b] = f->batch;
            if ((r->tcp_flags & (TCP_FIN | TCP_RST)) && !s->ended) {
                s->ended = 1; /* end_time = now, src/packets.rs:192-197, 422-426 */
                s->rec.end_seen = pos;
                s->rec.conn_state = conn_state_of(s->hist, s->hist_len, s->conn_state);
                s->rec.end_mask = (uint8_t)(s->rec.hist_mask & 0xFFu);
            }
        }
        s->rec.last_seen = pos; /* last_activity, src/packets.rs:184 */
    }
}

uint64_t orc_flows_count(const orc_flows* f) { return f->count; }

uint64_t orc_flows_export_times(const orc_flows* f, fb_flow_time* out, double* ref_f64, uint64_t cap) {
    /* in the order of orc_flows_export_sorted (derived Ord of the keys) */
    fb_flow_rec* recs = (fb_flow_rec*)malloc((f->count ? f->count : 1) * sizeof(fb_flow_rec));
    const uint64_t m = orc_flows_export_sorted(f, recs, f->count);
    uint64_t k = 0;
    for (; k < m && k < cap; ++k) {
        const orc_flow* s = find_slot(f->slots, f->cap, &recs[k].key);
        out[k] = s->tm;
        out[k].slot = 0;
        if (ref_f64) {
            ref_f64[2 * k] = s->ref_total_s;
            ref_f64[2 * k + 1] = s->ref_ia_s;
        }
    }
    free(recs);
    return k;
}

static int ip_cmp(uint32_t fam, const uint32_t* a, const uint32_t* b) {
    int nw = fam == 2 ? 1 : 4;
    for (int k = 0; k < nw; ++k)
        if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    return 0;
}

int orc_key_cmp(const fb_session_key* a, const fb_session_key* b) {
    if (a->protocol != b->protocol) return a->protocol < b->protocol ? -1 : 1; /* TCP < UDP */
    if (a->family != b->family) return a->family < b->family ? -1 : 1;         /* V4 < V6 */
    int c = ip_cmp(a->family, a->src_ip, b->src_ip);
    if (c) return c;
    if (a->src_port != b->src_port) return a->src_port < b->src_port ? -1 : 1;
    c = ip_cmp(a->family, a->dst_ip, b->dst_ip);
    if (c) return c;
    if (a->dst_port != b->dst_port) return a->dst_port < b->dst_port ? -1 : 1;
    return 0;
}

static int rec_cmp(const void* x, const void* y) {
    return orc_key_cmp(&((const fb_flow_rec*)x)->key, &((const fb_flow_rec*)y)->key);
}

uint64_t orc_flows_export_sorted(const orc_flows* f, fb_flow_rec* out, uint64_t cap) {
    uint64_t m = 0;
    for (uint64_t i = 0; i < f->cap && m < cap; ++i)
        if (f->slots[i].used) out[m++] = f->slots[i].rec;
    qsort(out, m, sizeof(fb_flow_rec), rec_cmp);
    return m;
}

int64_t orc_flows_history(const orc_flows* f, const fb_session_key* key, char* buf, uint64_t cap,
                          char* cs, uint64_t cs_cap) {
    orc_flow* s = find_slot(f->slots, f->cap, key);
    if (!s->used) return -1;
    uint64_t m = s->hist_len < cap ? s->hist_len : cap;
    if (m) memcpy(buf, s->hist, m);
    if (cs && cs_cap) {
        if (s->ended) {
            strncpy(cs, s->conn_state, cs_cap - 1);
            cs[cs_cap - 1] = 0;
        } else {
            cs[0] = 0;
        }
    }
    return (int64_t)s->hist_len;
}

/* ---- multi-GPU session-table merge (restated for the tests; flodbadd_amd/csrc/fb_merge.hip is
 * the product).  W ranks each hold a table of their contiguous packet-index shards, update call k
 * of every rank being its shard of global batch k (global order: batch, then rank, then packet).
 * The merged table must equal ONE table fed the packets in global order (src/packets.rs:329-535):
 * counters sum, start = earliest, last_activity = latest, history = the ranks' strings interleaved
 * in global order -- so its length sums and its character set is the union -- and end_time /
 * conn_state are decided at the globally first FIN/RST packet over the characters present then.
 * ------------------------------------------------------------------------------------------- */

/* The library's key hash (fb_flow_hash, flodbadd_amd/csrc/fb_internal.h flow_hash_words): the merge
 * assigns each key to the owner rank ((hash >> 32) * world) >> 32. */
uint64_t orc_flow_hash(const fb_session_key* key) {
    uint32_t k[10];
    memcpy(k, key, 40);
    k[9] &= 0xFFFFu;
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int j = 0; j < 10; j += 2) {
        h ^= (uint64_t)k[j] | ((uint64_t)k[j + 1] << 32);
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    return h;
}

static uint32_t owner_of(const fb_session_key* k, uint32_t world) {
    return (uint32_t)(((orc_flow_hash(k) >> 32) * (uint64_t)world) >> 32);
}

/* A position (update call << 32 | pkt_index) made global: call k was this rank's shard of global
 * batch map[k] >> 32 starting at global packet map[k] & 0xFFFFFFFF (without a map: batch k, the
 * shard at shard_first). */
static uint64_t globalize(uint64_t pos, uint64_t shard_first, const uint64_t* map) {
    const uint64_t m = map ? map[pos >> 32] : ((pos & 0xFFFFFFFF00000000ull) | shard_first);
    return (m & 0xFFFFFFFF00000000ull) | ((m & 0xFFFFFFFFull) + (pos & 0xFFFFFFFFull));
}

static uint64_t export_merge(const orc_flows* f, uint32_t world, uint32_t rank, uint64_t shard_first,
                             const uint64_t* map, fb_flow_mrec* out, uint64_t* counts);

uint64_t orc_flows_export_merge(const orc_flows* f, uint32_t world, uint32_t rank, uint64_t shard_first,
                                fb_flow_mrec* out, uint64_t* counts) {
    return export_merge(f, world, rank, shard_first, NULL, out, counts);
}

uint64_t orc_flows_export_merge_map(const orc_flows* f, uint32_t world, uint32_t rank, const uint64_t* call_map,
                                    fb_flow_mrec* out, uint64_t* counts) {
    return export_merge(f, world, rank, 0, call_map, out, counts);
}

static uint64_t export_merge(const orc_flows* f, uint32_t world, uint32_t rank, uint64_t shard_first,
                             const uint64_t* map, fb_flow_mrec* out, uint64_t* counts) {
    /* the table in Ord order, then stably grouped by owner */
    const uint64_t n = f->count;
    fb_flow_rec* recs = (fb_flow_rec*)malloc((n ? n : 1) * sizeof(fb_flow_rec));
    uint32_t(*calls)[4] = (uint32_t(*)[4])malloc((n ? n : 1) * sizeof(uint32_t[4]));
    uint64_t m = orc_flows_export_sorted(f, recs, n);
    for (uint64_t i = 0; i < m; ++i) {
        orc_flow* s = find_slot(f->slots, f->cap, &recs[i].key);
        memcpy(calls[i], s->char_call, sizeof(calls[i]));
    }
    uint64_t w = 0;
    for (uint32_t o = 0; o < world; ++o) {
        counts[o] = 0;
        for (uint64_t i = 0; i < m; ++i) {
            if (owner_of(&recs[i].key, world) != o) continue;
            fb_flow_mrec* x = &out[w++];
            x->rec = recs[i];
            x->rec.first_seen = globalize(x->rec.first_seen, shard_first, map);
            x->rec.last_seen = globalize(x->rec.last_seen, shard_first, map);
            if (x->rec.end_seen != FB_SEEN_NONE) x->rec.end_seen = globalize(x->rec.end_seen, shard_first, map);
            x->rec.slot = rank;
            for (int b = 0; b < 4; ++b) /* the update call of the first S s H h -> its global batch */
                x->char_call[b] = (calls[i][b] == FB_CALL_NONE || !map) ? calls[i][b] : (uint32_t)(map[calls[i][b]] >> 32);
            counts[o]++;
        }
    }
    free(recs);
    free(calls);
    return w;
}

typedef struct { const fb_flow_mrec* r; uint64_t idx; } mref;
static int mref_cmp(const void* x, const void* y) {
    const mref *a = (const mref*)x, *b = (const mref*)y;
    int c = orc_key_cmp(&a->r->rec.key, &b->r->rec.key);
    if (c) return c;
    return a->idx < b->idx ? -1 : (a->idx > b->idx);
}
static int idx_cmp(const void* x, const void* y) {
    const uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
    return a < b ? -1 : (a > b);
}

uint64_t orc_flow_merge(const fb_flow_mrec* in, uint64_t n, fb_flow_rec* out) {
    mref* v = (mref*)malloc((n ? n : 1) * sizeof(mref));
    for (uint64_t i = 0; i < n; ++i) { v[i].r = &in[i]; v[i].idx = i; }
    qsort(v, n, sizeof(mref), mref_cmp);
    /* one merged record per run of equal keys, kept with the run's first input index */
    typedef struct { uint64_t first; fb_flow_rec rec; } merged;
    merged* mg = (merged*)malloc((n ? n : 1) * sizeof(merged));
    uint64_t nk = 0;
    for (uint64_t a = 0; a < n;) {
        uint64_t b = a + 1;
        while (b < n && orc_key_cmp(&v[a].r->rec.key, &v[b].r->rec.key) == 0) ++b;
        fb_flow_rec o = v[a].r->rec;
        uint64_t end = FB_SEEN_NONE;
        uint32_t r0 = 0;
        for (uint64_t i = a; i < b; ++i) { /* the globally first FIN/RST and its rank */
            const fb_flow_rec* x = &v[i].r->rec;
            if (x->end_seen < end) { end = x->end_seen; r0 = x->slot; }
        }
        o.outbound_bytes = o.inbound_bytes = o.orig_pkts = o.resp_pkts = o.orig_ip_bytes = o.resp_ip_bytes = 0;
        o.first_seen = FB_SEEN_NONE;
        o.last_seen = 0;
        o.hist_len = 0;
        o.hist_mask = 0;
        o.segment_count = 0;
        uint32_t present = 0; /* FB_HIST_CHARS bits present at the end packet */
        for (uint64_t i = a; i < b; ++i) {
            const fb_flow_mrec* x = v[i].r;
            o.outbound_bytes += x->rec.outbound_bytes;
            o.inbound_bytes += x->rec.inbound_bytes;
            o.orig_pkts += x->rec.orig_pkts;
            o.resp_pkts += x->rec.resp_pkts;
            o.orig_ip_bytes += x->rec.orig_ip_bytes;
            o.resp_ip_bytes += x->rec.resp_ip_bytes;
            /* the session keeps what its first packet's insert stored (src/packets.rs:429-466); the
               segment state follows its latest packet (src/packets.rs:151-159) */
            if (x->rec.first_seen < o.first_seen) { o.first_seen = x->rec.first_seen; o.session_flags = x->rec.session_flags; }
            if (x->rec.last_seen > o.last_seen) { o.last_seen = x->rec.last_seen; o.in_segment = x->rec.in_segment; }
            o.segment_count += x->rec.segment_count;
            o.hist_len += x->rec.hist_len;
            o.hist_mask |= x->rec.hist_mask;
            if (end == FB_SEEN_NONE) continue;
            if (x->rec.end_seen == end) { /* the ending rank: its characters at the end packet */
                present |= x->rec.end_mask;
            } else { /* another rank's S s H h that came before the end packet in global order */
                const uint32_t call_e = (uint32_t)(end >> 32);
                for (int k = 0; k < 4; ++k) {
                    const uint32_t c = x->char_call[k];
                    if (c != FB_CALL_NONE && (c < call_e || (c == call_e && x->rec.slot < r0))) present |= 1u << k;
                }
            }
        }
        o.end_seen = end;
        o.end_mask = 0;
        o.conn_state = FB_CONN_NONE;
        if (end != FB_SEEN_NONE) { /* determine_conn_state over a string holding those characters */
            char chars[16], cs[4];
            int nc = 0;
            for (int k = 0; k < 8; ++k)
                if (present & (1u << k)) chars[nc++] = FB_HIST_CHARS[k];
            o.conn_state = conn_state_of(chars, (uint64_t)nc, cs);
            o.end_mask = (uint8_t)present;
        }
        o.slot = 0;
        mg[nk].first = v[a].idx;
        mg[nk].rec = o;
        ++nk;
        a = b;
    }
    qsort(mg, nk, sizeof(merged), idx_cmp); /* (first is the leading u64 of each entry) */
    for (uint64_t i = 0; i < nk; ++i) out[i] = mg[i].rec;
    free(mg);
    free(v);
    return nk;
}

uint64_t orc_pipeline(const orc_cfg* c, orc_flows* fl, const uint8_t* frames, uint64_t fb,
                      const uint32_t* offsets, uint32_t n, fb_pkt_out* scratch,
                      fb_batch_stats* st) {
    uint32_t no = 0;
    orc_parse_classify(c, frames, fb, offsets, n, scratch, &no, NULL, NULL, NULL, st);
    if (fl) orc_flows_update(fl, scratch, no, st);
    return n;
}

/* ---------------------------------------------------------------------------------------
 * New-session enrichment (src/packets.rs:429-485): ASN (src/asn.rs:32-63, src/asn_db.rs:82-166)
 * and blacklists (src/blacklists.rs:205-260 is_ip_in_blacklist, 456-560 the session pass).
 * ------------------------------------------------------------------------------------- */
static int ip_cmp_fam(int v6, const uint32_t* a, const uint32_t* b) {
    for (int k = 0; k < (v6 ? 4 : 1); ++k)
        if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    return 0;
}

typedef struct { fb_asn_range r; uint32_t idx; int v6; } asn_sort_item;
static int asn_item_cmp(const void* x, const void* y) {
    const asn_sort_item* a = (const asn_sort_item*)x;
    const asn_sort_item* b = (const asn_sort_item*)y;
    int c = ip_cmp_fam(a->v6, a->r.start, b->r.start);
    if (!c) c = ip_cmp_fam(a->v6, a->r.end, b->r.end);
    if (!c) c = a->idx < b->idx ? -1 : (a->idx > b->idx ? 1 : 0); /* Vec::sort is stable */
    return c;
}

/* Db::from_tsv's filtering (start <= end) + `records.sort()` (src/asn_db.rs:111-137), in place;
 * returns the kept count. */
uint32_t orc_asn_prepare(fb_asn_range* recs, uint32_t n, uint32_t family) {
    const int v6 = family == 10;
    asn_sort_item* t = (asn_sort_item*)malloc((n ? n : 1) * sizeof(asn_sort_item));
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (ip_cmp_fam(v6, recs[i].start, recs[i].end) <= 0) {
            t[m].r = recs[i];
            t[m].idx = i;
            t[m].v6 = v6;
            ++m;
        }
    qsort(t, m, sizeof(asn_sort_item), asn_item_cmp);
    for (uint32_t i = 0; i < m; ++i) recs[i] = t[i].r;
    free(t);
    return m;
}

/* Db::lookup (src/asn_db.rs:144-166), literally: returns the record, or -1 for None. */
int32_t orc_asn_lookup(const fb_asn_range* recs, uint32_t n, uint32_t family, const uint32_t ip[4]) {
    const int v6 = family == 10;
    uint64_t low = 0, high = n;
    while (low < high) {
        const uint64_t mid = (low + high) / 2;
        const fb_asn_range* rec = &recs[mid];
        if (ip_cmp_fam(v6, rec->start, ip) <= 0 && ip_cmp_fam(v6, ip, rec->end) <= 0) return (int32_t)rec->record;
        if (ip_cmp_fam(v6, ip, rec->start) < 0) high = mid;
        else low = mid + 1;
    }
    return -1;
}

/* IpNet::contains(&IpAddr): same family and network() <= ip <= broadcast(). */
static int net_contains(const fb_cidr* c, uint32_t family, const uint32_t ip[4]) {
    if (c->family != family) return 0;
    const int words = family == 10 ? 4 : 1;
    for (int k = 0; k < words; ++k) {
        const int bits = (int)c->prefix - 32 * k;
        const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : 0xFFFFFFFFu << (32 - bits));
        if ((ip[k] & m) != (c->addr[k] & m)) return 0;
    }
    return 1;
}

/* For every list: does some range of it contain ip (is_ip_in_blacklist's linear scan). */
uint64_t orc_blacklist_mask(const fb_cidr* nets, uint32_t n, uint32_t family, const uint32_t ip[4]) {
    uint64_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (net_contains(&nets[i], family, ip)) m |= 1ull << nets[i].list;
    return m;
}

/* The per-new-session lookups for `nk` keys (slot = index).  The ASN tables must have been
 * through orc_asn_prepare. */
void orc_enrich_keys(const orc_cfg* c, const fb_asn_range* a4, uint32_t n4, const fb_asn_range* a6, uint32_t n6,
                     const fb_cidr* nets, uint32_t nn, const fb_session_key* keys, uint32_t nk,
                     fb_flow_enrich* out) {
    for (uint32_t i = 0; i < nk; ++i) {
        const fb_session_key* k = &keys[i];
        const uint32_t fam = k->family;
        const int ls = orc_is_lan_ip(c, fam, k->src_ip), ld = orc_is_lan_ip(c, fam, k->dst_ip);
        fb_flow_enrich* r = &out[i];
        memset(r, 0, sizeof(*r));
        r->slot = i;
        r->flags = (ls ? FB_ENRICH_LOCAL_SRC : 0) | (ld ? FB_ENRICH_LOCAL_DST : 0) |
                   (is_own_ip(c, fam, k->src_ip) ? FB_ENRICH_SELF_SRC : 0) |
                   (is_own_ip(c, fam, k->dst_ip) ? FB_ENRICH_SELF_DST : 0);
        const fb_asn_range* A = fam == 10 ? a6 : a4;
        const uint32_t na = fam == 10 ? n6 : n4;
        r->src_asn = ls ? -1 : orc_asn_lookup(A, na, fam, k->src_ip);
        r->dst_asn = ld ? -1 : orc_asn_lookup(A, na, fam, k->dst_ip);
        r->src_blacklists = ls ? 0 : orc_blacklist_mask(nets, nn, fam, k->src_ip);
        r->dst_blacklists = ld ? 0 : orc_blacklist_mask(nets, nn, fam, k->dst_ip);
    }
}

/* ---------------------------------------------------------------------------------------
 * DNS divert parse: dns_parser::Packet::parse (dns-parser 0.8.0, restated from its published
 * source; the crate is a git dependency absent from the reference mount -> parity unpinned) and
 * what process_dns_packet reads from it (src/dns.rs:35-99).  Written in the crate's slice style:
 * a Name is scanned over `data` (a suffix of the message or an RDATA slice) with pointers into
 * `original` (the whole message).
 * ------------------------------------------------------------------------------------- */
typedef struct { const uint8_t* p; uint32_t n; } dslice;

static uint32_t rd16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* Name::scan: returns an fb_dns_status; *byte_len as Name::byte_len(). */
static uint32_t dn_scan(dslice data, dslice original, uint32_t* byte_len) {
    dslice pd = data;
    size_t pos = 0;
    long return_pos = -1;
    if (pd.n <= pos) return FB_DNS_UNEXPECTED_EOF;
    size_t largest_pos = original.n;
    uint8_t byte = pd.p[pos];
    while (byte != 0) {
        if (pd.n <= pos) return FB_DNS_UNEXPECTED_EOF;
        if ((byte & 0xC0) == 0xC0) {
            if (pd.n < pos + 2) return FB_DNS_UNEXPECTED_EOF;
            size_t off = rd16(pd.p + pos) & 0x3FFF;
            if (off >= original.n) return FB_DNS_UNEXPECTED_EOF;
            if (return_pos < 0) return_pos = (long)pos;
            if (off >= largest_pos) return FB_DNS_BAD_POINTER;
            largest_pos = off;
            pos = 0;
            pd.p = original.p + off;
            pd.n = original.n - (uint32_t)off;
        } else if ((byte & 0xC0) == 0) {
            size_t end = pos + byte + 1;
            if (pd.n < end) return FB_DNS_UNEXPECTED_EOF;
            for (size_t k = pos + 1; k < end; ++k)
                if (pd.p[k] & 0x80) return FB_DNS_LABEL_NOT_ASCII;
            pos = end;
            if (pd.n <= pos) return FB_DNS_UNEXPECTED_EOF;
        } else {
            return FB_DNS_UNKNOWN_LABEL_FORMAT;
        }
        byte = pd.p[pos];
    }
    *byte_len = return_pos >= 0 ? (uint32_t)return_pos + 2 : (uint32_t)pos + 1;
    return FB_DNS_OK;
}

/* Name's Display, recursively as the crate writes it. */
static void dn_fmt(const uint8_t* labels, dslice original, char* out, size_t* n) {
    size_t pos = 0;
    for (;;) {
        uint8_t byte = labels[pos];
        if (byte == 0) return;
        if ((byte & 0xC0) == 0xC0) {
            size_t off = rd16(labels + pos) & 0x3FFF;
            if (pos != 0) out[(*n)++] = '.';
            dn_fmt(original.p + off, original, out, n);
            return;
        }
        if (pos != 0) out[(*n)++] = '.';
        memcpy(out + *n, labels + pos + 1, byte);
        *n += byte;
        pos += byte + 1;
    }
}

static int qtype_ok(uint32_t t) { return (t >= 1 && t <= 16 && t != 3) || t == 28 || t == 33 || (t >= 252 && t <= 255); }
static int type_ok(uint32_t t) { return (t >= 1 && t <= 16 && t != 3) || t == 28 || t == 33 || t == 41 || t == 47; }

/* RData::parse for the types the crate decodes (others: RData::Unknown, never an error). */
static uint32_t rdata_parse(uint32_t typ, dslice rd, dslice original) {
    uint32_t bl, b2;
    switch (typ) {
        case 1: return rd.n == 4 ? FB_DNS_OK : FB_DNS_WRONG_RDATA_LENGTH;
        case 28: return rd.n == 16 ? FB_DNS_OK : FB_DNS_WRONG_RDATA_LENGTH;
        case 2: case 5: case 12: return dn_scan(rd, original, &bl);
        case 15: {
            if (rd.n < 3) return FB_DNS_WRONG_RDATA_LENGTH;
            dslice s = {rd.p + 2, rd.n - 2};
            return dn_scan(s, original, &bl);
        }
        case 33: {
            if (rd.n < 7) return FB_DNS_WRONG_RDATA_LENGTH;
            dslice s = {rd.p + 6, rd.n - 6};
            return dn_scan(s, original, &bl);
        }
        case 6: {
            uint32_t st = dn_scan(rd, original, &bl);
            if (st) return st;
            dslice s = {rd.p + bl, rd.n - bl};
            st = dn_scan(s, original, &b2);
            if (st) return st;
            return rd.n - bl - b2 < 20 ? FB_DNS_WRONG_RDATA_LENGTH : FB_DNS_OK;
        }
        case 16: {
            if (rd.n < 1) return FB_DNS_WRONG_RDATA_LENGTH;
            size_t pos = 0;
            while (pos < rd.n) {
                size_t l = rd.p[pos];
                pos += 1;
                if (rd.n < l + pos) return FB_DNS_WRONG_RDATA_LENGTH;
                pos += l;
            }
            return FB_DNS_OK;
        }
        default: return FB_DNS_OK;
    }
}

/* parse_record; answers' A / AAAA collected into addrs. */
static uint32_t parse_record(dslice data, size_t* offset, int answer, fb_ip* addrs, uint32_t* na, uint32_t* flags) {
    uint32_t bl;
    dslice s = {data.p + *offset, data.n - (uint32_t)*offset};
    uint32_t st = dn_scan(s, data, &bl);
    if (st) return st;
    *offset += bl;
    if (*offset + 10 > data.n) return FB_DNS_UNEXPECTED_EOF;
    uint32_t typ = rd16(data.p + *offset);
    if (!type_ok(typ)) return FB_DNS_INVALID_TYPE;
    *offset += 2;
    uint32_t cls = rd16(data.p + *offset);
    if (typ != 41 && !((cls & 0x7FFF) >= 1 && (cls & 0x7FFF) <= 4)) return FB_DNS_INVALID_CLASS;
    *offset += 2 + 4; /* class, ttl */
    size_t rdlen = rd16(data.p + *offset);
    *offset += 2;
    if (*offset + rdlen > data.n) return FB_DNS_UNEXPECTED_EOF;
    dslice rd = {data.p + *offset, (uint32_t)rdlen};
    st = rdata_parse(typ, rd, data);
    if (st) return st;
    if (answer && (typ == 1 || typ == 28)) {
        if (*na < FB_DNS_MAX_ADDRS) {
            fb_ip* a = &addrs[(*na)++];
            memset(a, 0, sizeof(*a));
            a->family = typ == 28 ? 10 : 2;
            for (int k = 0; k < (typ == 28 ? 4 : 1); ++k) a->addr[k] = be32(rd.p + 4 * k);
        } else {
            *flags |= FB_DNS_ADDRS_TRUNCATED;
        }
    }
    *offset += rdlen;
    return FB_DNS_OK;
}

static int ends_with(const char* s, size_t n, const char* sfx) {
    size_t l = strlen(sfx);
    return n >= l && memcmp(s + n - l, sfx, l) == 0;
}

/* Packet::parse + the fields process_dns_packet reads. name: >= FB_DNS_MAX_NAME bytes. */
uint32_t orc_dns_parse(const uint8_t* payload, uint32_t len, uint32_t pkt_index, fb_dns_msg* r, char* name,
                       fb_ip* addrs) {
    memset(r, 0, sizeof(*r));
    r->pkt_index = pkt_index;
    dslice data = {payload, len};
    uint32_t st = FB_DNS_OK, flags = 0, na = 0;
    if (len < 12) {
        r->status = FB_DNS_HEADER_TOO_SHORT;
        return r->status;
    }
    r->id = (uint16_t)rd16(payload);
    uint32_t qd = rd16(payload + 4), an = rd16(payload + 6), ns = rd16(payload + 8), ar = rd16(payload + 10);
    r->questions = (uint16_t)qd;
    r->answers = (uint16_t)an;
    if ((payload[2] & 0x80) == 0) flags |= FB_DNS_QUERY;
    size_t offset = 12, q0 = 0;
    for (uint32_t q = 0; q < qd && !st; ++q) {
        uint32_t bl;
        dslice s = {payload + offset, len - (uint32_t)offset};
        st = dn_scan(s, data, &bl);
        if (st) break;
        if (q == 0) q0 = offset;
        offset += bl;
        if (offset + 4 > len) { st = FB_DNS_UNEXPECTED_EOF; break; }
        if (!qtype_ok(rd16(payload + offset))) { st = FB_DNS_INVALID_QUERY_TYPE; break; }
        offset += 2;
        uint32_t qc = rd16(payload + offset) & 0x7FFF;
        if (!((qc >= 1 && qc <= 4) || qc == 255)) { st = FB_DNS_INVALID_QUERY_CLASS; break; }
        offset += 2;
    }
    for (uint32_t k = 0; k < an && !st; ++k) st = parse_record(data, &offset, 1, addrs, &na, &flags);
    for (uint32_t k = 0; k < ns && !st; ++k) st = parse_record(data, &offset, 0, addrs, &na, &flags);
    int have_opt = 0;
    for (uint32_t k = 0; k < ar && !st; ++k) {
        if (offset + 3 <= len && payload[offset] == 0 && payload[offset + 1] == 0 && payload[offset + 2] == 41) {
            offset += 1;
            if (have_opt) { st = FB_DNS_ADDITIONAL_OPT; break; }
            have_opt = 1;
            if (offset + 10 > len) { st = FB_DNS_UNEXPECTED_EOF; break; } /* parse_opt_record */
            offset += 8;
            size_t rdlen = rd16(payload + offset);
            offset += 2;
            if (offset + rdlen > len) { st = FB_DNS_UNEXPECTED_EOF; break; }
            offset += rdlen;
        } else {
            st = parse_record(data, &offset, 0, addrs, &na, &flags);
        }
    }
    r->status = (uint8_t)st;
    if (st) return st;
    if (qd > 0) {
        char* full = (char*)malloc(len * 2 + 16); /* a scanned name's Display is bounded by the message */
        size_t n = 0;
        dn_fmt(payload + q0, data, full, &n);
        flags |= FB_DNS_HAS_QUESTION;
        if (ends_with(full, n, ".in-addr.arpa") || ends_with(full, n, ".ip6.arpa")) flags |= FB_DNS_REVERSE;
        if (n > FB_DNS_MAX_NAME - 1) flags |= FB_DNS_NAME_TRUNCATED;
        r->name_len = (uint16_t)(n < FB_DNS_MAX_NAME - 1 ? n : FB_DNS_MAX_NAME - 1);
        memcpy(name, full, r->name_len);
        free(full);
    }
    r->flags = (uint8_t)flags;
    r->n_addrs = (uint8_t)na;
    return FB_DNS_OK;
}

/* ---------------------------------------------------------------------------------------
 * All-cores CPU baseline: the batch split into `threads` contiguous ranges,
 * each parsed + classified by orc_parse_classify into a thread-local region, then compacted into
 * packet order.  Same outputs as one orc_parse_classify over the batch (checked in tests).
 * ------------------------------------------------------------------------------------- */
#ifdef _OPENMP
#include <omp.h>
#endif
int orc_parse_classify_mt(const orc_cfg* c, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                          uint32_t n, fb_pkt_out* out, uint32_t* n_out, fb_dns_out* dns, uint32_t* n_dns,
                          fb_batch_stats* st, int threads) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n) threads = n ? (int)n : 1;
    uint32_t cs[256], cd[256];
    fb_batch_stats ts[256];
    if (threads > 256) threads = 256;
#pragma omp parallel for num_threads(threads) schedule(static, 1)
    for (int t = 0; t < threads; ++t) {
        const uint32_t a = (uint32_t)((uint64_t)n * t / threads), b = (uint32_t)((uint64_t)n * (t + 1) / threads);
        /* frames [a, b): offsets stay absolute, pkt_index relative -> fixed below */
        orc_parse_classify(c, frames, frames_bytes, offsets + a, b - a, out + a, &cs[t], dns + a, &cd[t], NULL, &ts[t]);
        for (uint32_t k = 0; k < cs[t]; ++k) out[a + k].pkt_index += a;
        for (uint32_t k = 0; k < cd[t]; ++k) dns[a + k].pkt_index += a;
    }
    /* compaction into packet order + stats merge */
    uint32_t so = 0, sd = 0;
    fb_batch_stats m;
    memset(&m, 0, sizeof(m));
    for (int t = 0; t < threads; ++t) {
        const uint32_t a = (uint32_t)((uint64_t)n * t / threads);
        if (so != a) memmove(out + so, out + a, (size_t)cs[t] * sizeof(fb_pkt_out));
        if (sd != a) memmove(dns + sd, dns + a, (size_t)cd[t] * sizeof(fb_dns_out));
        so += cs[t];
        sd += cd[t];
        uint64_t* dst = (uint64_t*)&m;
        const uint64_t* src = (const uint64_t*)&ts[t];
        for (size_t k = 0; k < sizeof(m) / 8; ++k) dst[k] += src[k];
    }
    if (n_out) *n_out = so;
    if (n_dns) *n_dns = sd;
    if (st) *st = m;
    return 0;
}

/* ---------------------------------------------------------------------------------------
 * All-cores parse + session-table baseline (SURVEY.md 8d (ii) for config C4): parse + classify in
 * `threads` contiguous ranges (orc_parse_classify_mt), then the SESSION records are split by an
 * owner thread taken from their key hash (a stable counting sort, so each owner sees its records
 * in packet order) and every thread upserts its own keys into its own table.  A key's records
 * all go to one table in batch order, so the union of the tables is exactly the single-thread
 * table (checked in tests).  Returns the number of SESSION records.
 * ------------------------------------------------------------------------------------- */
uint64_t orc_pipeline_mt(const orc_cfg* c, orc_flows** tables, int threads, const uint8_t* frames, uint64_t fb,
                         const uint32_t* offsets, uint32_t n, fb_pkt_out* scratch, fb_dns_out* dns_scratch,
                         fb_batch_stats* st) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint32_t no = 0, nd = 0;
    fb_batch_stats s;
    orc_parse_classify_mt(c, frames, fb, offsets, n, scratch, &no, dns_scratch, &nd, &s, threads);
    const int T = threads;
    uint32_t* own = (uint32_t*)malloc((size_t)(no ? no : 1) * 4);
    uint32_t* idx = (uint32_t*)malloc((size_t)(no ? no : 1) * 4);
    uint64_t* cnt = (uint64_t*)calloc((size_t)T * T, 8); /* cnt[range * T + owner] -> scatter cursor */
    uint64_t* beg = (uint64_t*)calloc((size_t)T + 1, 8);
    fb_batch_stats ts[256];
#pragma omp parallel num_threads(T)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        const uint32_t a = (uint32_t)((uint64_t)no * t / T), b = (uint32_t)((uint64_t)no * (t + 1) / T);
        for (uint32_t i = a; i < b; ++i) {
            own[i] = (uint32_t)((key_hash(&scratch[i].key) >> 40) % (uint64_t)T);
            cnt[(size_t)t * T + own[i]]++;
        }
#pragma omp barrier
#pragma omp single
        {
            uint64_t run = 0;
            for (int o = 0; o < T; ++o) {
                beg[o] = run;
                for (int r = 0; r < T; ++r) {
                    const uint64_t k = cnt[(size_t)r * T + o];
                    cnt[(size_t)r * T + o] = run;
                    run += k;
                }
            }
            beg[T] = run;
        }
        for (uint32_t i = a; i < b; ++i) idx[cnt[(size_t)t * T + own[i]]++] = i;
#pragma omp barrier
        memset(&ts[t], 0, sizeof(ts[t]));
        for (uint64_t k = beg[t]; k < beg[t + 1]; ++k) flow_upsert(tables[t], &scratch[idx[k]], &ts[t], NULL);
        tables[t]->batch++;
    }
    for (int t = 0; t < T; ++t) {
        s.new_sessions += ts[t].new_sessions;
        s.updated_sessions += ts[t].updated_sessions;
    }
    free(own);
    free(idx);
    free(cnt);
    free(beg);
    if (st) *st = s;
    return no;
}
