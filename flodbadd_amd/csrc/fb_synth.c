/*
 * fb_synth.c -- deterministic synthetic capture batches, for tests and bench.
 *
 * Frames are Ethernet/IPv4|IPv6/TCP|UDP with consistent length fields (IPv4 total_length =
 * caplen - 14, IPv6 payload_length = caplen - 54), packed back to back with u32 offsets --
 * the buffer a libpcap capture loop would hand the reference one frame at a time
 * (src/capture.rs:1088-1092).  Every value is a pure function of (seed, flow id, global packet
 * index), so a batch can be generated in parallel and any shard [first, first+n) of a larger
 * virtual batch is reproducible on its own (multi-GPU sharding by packet index).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct fb_synth_cfg {
    uint64_t seed;         /* 0xF10DBADD ^ config_id */
    uint32_t n_flows;      /* flow pool size F */
    uint32_t mode;         /* 0: all 64-B IPv4/TCP (C2); 1: IMIX 64/576/1500 7:4:1 (C3/C4) */
    uint32_t v6_permille;  /* IMIX only: IPv6 share (200) */
    uint32_t udp_permille; /* IMIX only: UDP share (300) */
    uint32_t dns_permille; /* flows on port 53 (5) */
    uint32_t zipf;         /* 0 uniform flow choice, 1 Zipf(s) */
    double zipf_s;         /* 1.1 */
    uint32_t lan_dst_permille; /* flows whose dst is a LAN address too (0: SURVEY.md §8d's mix, every
                                  dst public); with a LAN src (50 %) such a flow is local, so the
                                  Local/Global filters drop a large share (filter parity tests) */
} fb_synth_cfg;

static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t mix(uint64_t a, uint64_t b) {
    uint64_t s = a ^ (b * 0xD6E8FEB86659FD93ull);
    return splitmix64(&s);
}
static uint32_t below(uint64_t* s, uint32_t n) { return (uint32_t)((splitmix64(s) >> 32) * n >> 32); }

typedef struct flow {
    uint32_t src[4], dst[4];
    uint16_t sport, dport;
    uint8_t v6, udp;
} flow;

static int lan_v4(uint32_t v) {
    uint32_t a = v >> 24, b = (v >> 16) & 0xff;
    return v == 0 || v == 0xffffffffu || a == 127 || (v >> 28) == 0xE || (v >> 16) == 0xA9FE || a == 10 ||
           (a == 172 && b >= 16 && b <= 31) || (v >> 16) == 0xC0A8;
}

static uint32_t public_v4(uint64_t* s) {
    for (;;) {
        uint32_t v = (uint32_t)(splitmix64(s) >> 32);
        uint32_t a = v >> 24;
        if (a >= 1 && a <= 223 && !lan_v4(v)) return v;
    }
}

static const uint16_t kServicePorts[8] = {80, 443, 22, 8080, 3389, 5353, 123, 12345};

static void make_flow(const fb_synth_cfg* c, uint32_t f, flow* o) {
    uint64_t s = mix(c->seed ^ 0x5EED0F10ull, f);
    memset(o, 0, sizeof(*o));
    if (c->mode == 1) {
        o->v6 = below(&s, 1000) < c->v6_permille;
        o->udp = below(&s, 1000) < c->udp_permille;
    }
    int lan_src = below(&s, 2) == 0;
    if (!o->v6) {
        o->src[0] = lan_src ? (0x0A000000u | (uint32_t)(splitmix64(&s) >> 40)) : public_v4(&s);
        o->dst[0] = public_v4(&s);
    } else {
        /* LAN: fd00::/8 (unique local, src/ip.rs:127-129); public: 2000::/3 */
        for (int k = 0; k < 4; ++k) {
            o->src[k] = (uint32_t)(splitmix64(&s) >> 32);
            o->dst[k] = (uint32_t)(splitmix64(&s) >> 32);
        }
        o->src[0] = lan_src ? (0xFD000000u | (o->src[0] & 0x00FFFFFFu)) : (0x20000000u | (o->src[0] & 0x1FFFFFFFu));
        o->dst[0] = 0x20000000u | (o->dst[0] & 0x1FFFFFFFu);
    }
    if (c->lan_dst_permille) { /* its own stream: the mix above is unchanged */
        uint64_t t = mix(c->seed ^ 0x1A4D57ull, f);
        if (below(&t, 1000) < c->lan_dst_permille) {
            uint32_t r = (uint32_t)(splitmix64(&t) >> 32);
            if (!o->v6) /* 192.168/16 or 10/8 */
                o->dst[0] = (r & 1) ? (0xC0A80000u | (r >> 16)) : (0x0A000000u | (r >> 8));
            else        /* fe80::/10 or fd00::/8 */
                o->dst[0] = (r & 1) ? (0xFE800000u | ((r >> 8) & 0x003FFFFFu)) : (0xFD000000u | (r >> 8));
        }
    }
    o->sport = (uint16_t)(32768 + below(&s, 61000 - 32768));
    if (below(&s, 1000) < c->dns_permille) {
        o->dport = 53;
    } else if (below(&s, 10) < 6) {
        o->dport = kServicePorts[below(&s, 8)];
    } else {
        o->dport = (uint16_t)(32768 + below(&s, 61000 - 32768));
    }
}

/* Zipf inverse CDF over [0, F): cumulative weights k^-s, normalised.  Built once per call. */
static double* zipf_cdf(uint32_t F, double s) {
    double* c = (double*)malloc(sizeof(double) * F);
    if (!c) return NULL;
    double acc = 0;
    for (uint32_t k = 0; k < F; ++k) {
        acc += pow((double)(k + 1), -s);
        c[k] = acc;
    }
    for (uint32_t k = 0; k < F; ++k) c[k] /= acc;
    return c;
}
static uint32_t zipf_pick(const double* cdf, uint32_t F, double u) {
    uint32_t lo = 0, hi = F - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < u) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static uint32_t frame_len(const fb_synth_cfg* c, uint64_t pkt, const flow* fl) {
    if (c->mode == 0) return 64;
    uint64_t s = mix(c->seed ^ 0x1E11ull, pkt);
    uint32_t r = below(&s, 12); /* IMIX 7:4:1 */
    uint32_t L = r < 7 ? 64u : (r < 11 ? 576u : 1500u);
    if (L == 64 && fl->v6 && !fl->udp) L = 78; /* v6/TCP needs 74 B of headers */
    return L;
}

static uint32_t pick_flow(const fb_synth_cfg* c, const double* cdf, uint64_t pkt) {
    uint64_t s = mix(c->seed ^ 0xF10Full, pkt);
    if (c->zipf && cdf) {
        double u = (double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
        return zipf_pick(cdf, c->n_flows, u);
    }
    return below(&s, c->n_flows);
}

static void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* TCP flags distribution: SYN .05, SYN|ACK .05, ACK .55, PSH|ACK .30, FIN|ACK .04, RST .01 */
static uint8_t pick_flags(uint64_t* s) {
    uint32_t r = below(s, 100);
    if (r < 5) return 0x02;
    if (r < 10) return 0x12;
    if (r < 65) return 0x10;
    if (r < 95) return 0x18;
    if (r < 99) return 0x11;
    return 0x04;
}

static void write_frame(const fb_synth_cfg* c, uint64_t pkt, const flow* fl, uint8_t* f, uint32_t L) {
    uint64_t s = mix(c->seed ^ 0xFAA3ull, pkt);
    int rev = below(&s, 2) == 0; /* direction reversed 50 % */
    const uint32_t* sip = rev ? fl->dst : fl->src;
    const uint32_t* dip = rev ? fl->src : fl->dst;
    uint16_t sp = rev ? fl->dport : fl->sport, dp = rev ? fl->sport : fl->dport;
    /* Ethernet: dst/src MAC from the flow, ethertype */
    for (int k = 0; k < 6; ++k) { f[k] = (uint8_t)(0x02 + k); f[6 + k] = (uint8_t)(0x10 + k); }
    uint32_t l4;
    if (!fl->v6) {
        put16(f + 12, 0x0800);
        uint8_t* ip = f + 14;
        ip[0] = 0x45; ip[1] = 0;
        put16(ip + 2, L - 14);
        put16(ip + 4, (uint32_t)(pkt & 0xffff)); put16(ip + 6, 0x4000);
        ip[8] = 64; ip[9] = fl->udp ? 17 : 6;
        put16(ip + 10, 0);
        put32(ip + 12, sip[0]); put32(ip + 16, dip[0]);
        l4 = 34;
    } else {
        put16(f + 12, 0x86DD);
        uint8_t* ip = f + 14;
        put32(ip, 0x60000000u);
        put16(ip + 4, L - 54);
        ip[6] = fl->udp ? 17 : 6; ip[7] = 64;
        for (int k = 0; k < 4; ++k) { put32(ip + 8 + 4 * k, sip[k]); put32(ip + 24 + 4 * k, dip[k]); }
        l4 = 54;
    }
    uint8_t* t = f + l4;
    put16(t, sp); put16(t + 2, dp);
    uint32_t hdr;
    if (!fl->udp) {
        put32(t + 4, (uint32_t)splitmix64(&s)); put32(t + 8, (uint32_t)splitmix64(&s));
        t[12] = 0x50; t[13] = pick_flags(&s);
        put16(t + 14, 0xFFFF); put16(t + 16, 0); put16(t + 18, 0);
        hdr = l4 + 20;
    } else {
        put16(t + 4, L - l4); put16(t + 6, 0);
        hdr = l4 + 8;
    }
    /* payload: cheap deterministic filler (never read by the parser) */
    for (uint32_t i = hdr; i < L; ++i) f[i] = (uint8_t)(i * 31u + (uint32_t)pkt);
}

/* Fill offsets[0..n] for packets [first, first+n); returns the total byte count. */
uint64_t fb_synth_plan(const fb_synth_cfg* c, uint64_t first, uint32_t n, uint32_t* offsets) {
    double* cdf = c->zipf ? zipf_cdf(c->n_flows, c->zipf_s) : NULL;
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        flow fl;
        make_flow(c, pick_flow(c, cdf, first + i), &fl);
        offsets[i] = (uint32_t)off;
        off += frame_len(c, first + i, &fl);
    }
    offsets[n] = (uint32_t)off;
    free(cdf);
    return off;
}

/* Write the frames planned by fb_synth_plan into `frames` (sized offsets[n]).  Threads split
 * the packet range; results do not depend on n_threads. */
int fb_synth_fill(const fb_synth_cfg* c, uint64_t first, uint32_t n, const uint32_t* offsets, uint8_t* frames,
                  int n_threads) {
    double* cdf = c->zipf ? zipf_cdf(c->n_flows, c->zipf_s) : NULL;
    (void)n_threads;
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        flow fl;
        make_flow(c, pick_flow(c, cdf, first + (uint64_t)i), &fl);
        write_frame(c, first + (uint64_t)i, &fl, frames + offsets[i], offsets[i + 1] - offsets[i]);
    }
    free(cdf);
    return 0;
}

/* The flow a packet was drawn from (for test-side bookkeeping). */
uint32_t fb_synth_flow_of(const fb_synth_cfg* c, uint64_t pkt) {
    double* cdf = c->zipf ? zipf_cdf(c->n_flows, c->zipf_s) : NULL;
    uint32_t f = pick_flow(c, cdf, pkt);
    free(cdf);
    return f;
}
