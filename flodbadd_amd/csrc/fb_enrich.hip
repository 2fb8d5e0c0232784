// fb_enrich.hip -- new-session enrichment on the GPU.
//
// When process_parsed_packet inserts a session it computes, per new flow (src/packets.rs:429-485):
//   is_local_src/dst = is_lan_ip(key ip), is_self_src/dst = own_ips.contains(key ip),
//   src/dst ASN     = get_asn(ip) for non-local ips (src/asn.rs:32-63 -> Db::lookup,
//                     src/asn_db.rs:144-166: a binary search over ranges sorted by (start, end)),
// and the blacklist pass evaluates every non-local session ip against every range of every list
// (recompute_blacklist_for_sessions, src/blacklists.rs:456-560, is_ip_in_blacklist 205-260:
// IpNet::contains in a linear scan).  Here:
//   k_flow_enrich  one lane per table slot; flows of the table (or only those the last update
//                  inserted) get their flags, both ASN records and both blacklist masks, and are
//                  compacted into the output with a ballot + one atomic per block;
//   k_ip_lookup    the same lookups for an arbitrary address list (get_asn / is_ip_blacklisted).
// ASN: the exact probe sequence of Db::lookup (same mid, same comparisons), so even overlapping
// ranges give the reference's answer.  Blacklists: the host flattens the lists into disjoint
// elementary intervals with the set of lists covering each (an interval sweep,
// build_blacklist_tables below), so a lookup is one binary search instead of a scan of every
// range; "some range of list l contains ip" is unchanged.
#include <algorithm>
#include <vector>

#include "fb_internal.h"

namespace fbk {

// a < b over session_key ip words (word 0 most significant); v4 uses word 0 only
__device__ __forceinline__ bool ip_lt(const uint32_t a[4], const uint32_t b[4], bool v6) {
    if (!v6) return a[0] < b[0];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (a[k] != b[k]) return a[k] < b[k];
    return false;
}

// Db::lookup, src/asn_db.rs:144-166 -- returns the record, or -1 for None.
__device__ __forceinline__ int32_t asn_lookup(const fb_asn_range* T, uint32_t n, const uint32_t ip[4], bool v6) {
    uint32_t low = 0u, high = n;
    while (low < high) {
        const uint32_t mid = (low + high) >> 1;
        const fb_asn_range& r = T[mid];
        const bool ge_start = !ip_lt(ip, r.start, v6), le_end = !ip_lt(r.end, ip, v6);
        if (ge_start && le_end) return (int32_t)r.record;
        if (!ge_start) high = mid;
        else low = mid + 1u;
    }
    return -1;
}

// Lists whose ranges contain ip: the mask of the last elementary interval starting <= ip.
__device__ __forceinline__ unsigned long long bl_lookup(const EnrichTables& t, const uint32_t ip[4], bool v6) {
    uint32_t lo = 0u, hi = v6 ? t.m6 : t.m4;  // first interval starting > ip
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        bool gt;
        if (v6) {
            const uint4 p = t.bl6_pos[mid];
            const uint32_t pw[4] = {p.x, p.y, p.z, p.w};
            gt = ip_lt(ip, pw, true);
        } else {
            gt = ip[0] < t.bl4_pos[mid];
        }
        if (gt) hi = mid;
        else lo = mid + 1u;
    }
    if (lo == 0u) return 0ull;
    return v6 ? t.bl6_mask[lo - 1u] : t.bl4_mask[lo - 1u];
}

// The four lookups of a new flow (ASN and blacklist mask of src and dst) as independent searches
// advanced in one loop, so each step issues up to four loads together: the binary searches are
// chains of dependent loads (latency-bound), and interleaving them keeps 4x the loads in flight.
// Same probes as asn_lookup / bl_lookup.  A local ip (`skip`) gets -1 / 0 without a search.
__device__ __forceinline__ void flow_lookups(const EnrichTables& t, bool v6, const uint32_t* const ip[2],
                                             const bool skip[2], int32_t asn[2], unsigned long long bl[2]) {
    const fb_asn_range* A = v6 ? t.asn6 : t.asn4;
    const uint32_t na = v6 ? t.n6 : t.n4, nb = v6 ? t.m6 : t.m4;
    uint32_t alo[2], ahi[2], blo[2], bhi[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        alo[k] = 0u;
        ahi[k] = skip[k] ? 0u : na;
        blo[k] = 0u;
        bhi[k] = skip[k] ? 0u : nb;
        asn[k] = -1;
    }
    for (;;) {
        bool on_a[2], on_b[2];
        uint4 st[2], en[2], bp[2];
        uint32_t am[2], bm[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // issue every active search's probe
            on_a[k] = alo[k] < ahi[k];
            on_b[k] = blo[k] < bhi[k];
            am[k] = (alo[k] + ahi[k]) >> 1;
            bm[k] = (blo[k] + bhi[k]) >> 1;
            if (on_a[k]) {
                st[k] = *reinterpret_cast<const uint4*>(A[am[k]].start);
                en[k] = *reinterpret_cast<const uint4*>(A[am[k]].end);
            }
            if (on_b[k]) bp[k] = v6 ? t.bl6_pos[bm[k]] : make_uint4(t.bl4_pos[bm[k]], 0u, 0u, 0u);
        }
        if (!(on_a[0] || on_a[1] || on_b[0] || on_b[1])) break;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (on_a[k]) {  // Db::lookup, src/asn_db.rs:144-166
                const uint32_t sw[4] = {st[k].x, st[k].y, st[k].z, st[k].w}, ew[4] = {en[k].x, en[k].y, en[k].z, en[k].w};
                const bool ge_start = !ip_lt(ip[k], sw, v6), le_end = !ip_lt(ew, ip[k], v6);
                if (ge_start && le_end) {
                    asn[k] = (int32_t)A[am[k]].record;
                    ahi[k] = alo[k];  // found: the search ends
                } else if (!ge_start) {
                    ahi[k] = am[k];
                } else {
                    alo[k] = am[k] + 1u;
                }
            }
            if (on_b[k]) {  // first interval starting > ip
                const uint32_t pw[4] = {bp[k].x, bp[k].y, bp[k].z, bp[k].w};
                if (v6 ? ip_lt(ip[k], pw, true) : ip[k][0] < pw[0]) bhi[k] = bm[k];
                else blo[k] = bm[k] + 1u;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        bl[k] = 0ull;
        if (!skip[k] && blo[k] > 0u) bl[k] = v6 ? t.bl6_mask[blo[k] - 1u] : t.bl4_mask[blo[k] - 1u];
    }
}

__global__ __launch_bounds__(256) void k_ip_lookup(const EnrichTables t, const fb_ip* ips, uint32_t n, int32_t* asn,
                                                   unsigned long long* lists) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fb_ip x = ips[i];
    const bool v6 = x.family == 10u, ok = x.family == 2u || v6;
    if (asn) asn[i] = ok ? (v6 ? asn_lookup(t.asn6, t.n6, x.addr, true) : asn_lookup(t.asn4, t.n4, x.addr, false)) : -1;
    if (lists) lists[i] = ok ? bl_lookup(t, x.addr, v6) : 0ull;
}

__global__ __launch_bounds__(256) void k_flow_enrich(const EnrichTables t, const DevConfig* cfg, const FlowSlot* T,
                                                     unsigned long long cap, uint32_t new_only, uint32_t batch,
                                                     fb_flow_enrich* out, unsigned long long out_cap,
                                                     unsigned long long* d_n) {
    __shared__ unsigned long long sh[4];
    __shared__ unsigned long long s_base;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < cap; base += stride) {
        const unsigned long long i = base + threadIdx.x;
        bool take = i < cap && T[i].tag >= 2ull;
        if (take && new_only) take = (uint32_t)(T[i].first_seen >> 32) == batch;
        const unsigned long long m = __ballot(take);
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
        if (take && pos < out_cap) {
            const uint32_t* k = T[i].key;
            const uint32_t src[4] = {k[0], k[1], k[2], k[3]}, dst[4] = {k[4], k[5], k[6], k[7]};
            const uint32_t fam = (k[9] >> 8) & 0xFFu;
            const bool v6 = fam == 10u;
            // src/packets.rs:429-435 (the key as stored, i.e. canonical)
            const bool ls = v6 ? lan_v6(cfg, cfg, src) : lan_v4(src[0]);
            const bool ld = v6 ? lan_v6(cfg, cfg, dst) : lan_v4(dst[0]);
            fb_flow_enrich r;
            r.slot = (uint32_t)i;
            r.flags = (ls ? FB_ENRICH_LOCAL_SRC : 0u) | (ld ? FB_ENRICH_LOCAL_DST : 0u) |
                      (own_ip(cfg, cfg, fam, src) ? FB_ENRICH_SELF_SRC : 0u) |
                      (own_ip(cfg, cfg, fam, dst) ? FB_ENRICH_SELF_DST : 0u);
            // ASN only for non-local ips (src/packets.rs:468-485); so the blacklist ips
            // (src/blacklists.rs:545-556)
            const uint32_t* const ips[2] = {src, dst};
            const bool skip[2] = {ls, ld};
            int32_t asn[2];
            unsigned long long bl[2];
            flow_lookups(t, v6, ips, skip, asn, bl);
            r.src_asn = asn[0];
            r.dst_asn = asn[1];
            r.src_blacklists = bl[0];
            r.dst_blacklists = bl[1];
            out[pos] = r;
        }
        __syncthreads();
    }
}

hipError_t launch_ip_lookup(const EnrichTables& t, const fb_ip* ips, uint32_t n, int32_t* asn,
                            unsigned long long* lists, hipStream_t s) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(k_ip_lookup, dim3((n + 255u) / 256u), dim3(256), 0, s, t, ips, n, asn, lists);
    return hipGetLastError();
}

#ifndef FB_ENRICH_GRID
#define FB_ENRICH_GRID 8192ull  // one slot per thread up to 2^21 slots: 0.38 ms vs 0.43 at 2048 (C4)
#endif
hipError_t launch_flow_enrich(const EnrichTables& t, const DevConfig* cfg, const FlowSlot* table,
                              unsigned long long cap, uint32_t new_only, uint32_t batch, fb_flow_enrich* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > FB_ENRICH_GRID) g = FB_ENRICH_GRID;
    if (g == 0ull) g = 1ull;
    hipLaunchKernelGGL(k_flow_enrich, dim3((uint32_t)g), dim3(256), 0, s, t, cfg, table, cap, new_only, batch, out,
                       out_cap, d_n);
    return hipGetLastError();
}

// ---- host: blacklist interval tables ----------------------------------------------------------
namespace {
typedef unsigned __int128 u128;
u128 to128(const uint32_t w[4]) {
    return ((u128)w[0] << 96) | ((u128)w[1] << 64) | ((u128)w[2] << 32) | (u128)w[3];
}
struct Ev {
    u128 pos;
    uint32_t list;
    int delta;
};
// Sweep one family's [start, end] ranges into disjoint intervals with their covering lists.
void sweep(std::vector<Ev>& ev, std::vector<u128>& pos, std::vector<unsigned long long>& mask) {
    std::sort(ev.begin(), ev.end(), [](const Ev& a, const Ev& b) { return a.pos < b.pos; });
    uint32_t cnt[FB_MAX_BLACKLISTS] = {0};
    for (size_t i = 0; i < ev.size();) {
        const u128 p = ev[i].pos;
        for (; i < ev.size() && ev[i].pos == p; ++i) cnt[ev[i].list] += ev[i].delta;
        unsigned long long m = 0ull;
        for (uint32_t l = 0; l < FB_MAX_BLACKLISTS; ++l) m |= cnt[l] ? 1ull << l : 0ull;
        if (!mask.empty() && mask.back() == m) continue;  // same lists as the interval before
        pos.push_back(p);
        mask.push_back(m);
    }
}
}  // namespace

// Returns false on an invalid entry (family, prefix or list out of range).
bool build_blacklist_tables(const fb_cidr* nets, uint32_t n, std::vector<uint32_t>& p4,
                            std::vector<unsigned long long>& m4, std::vector<uint4>& p6,
                            std::vector<unsigned long long>& m6) {
    std::vector<Ev> e4, e6;
    for (uint32_t i = 0; i < n; ++i) {
        const fb_cidr& c = nets[i];
        const bool v6 = c.family == 10u;
        if ((c.family != 2u && !v6) || c.prefix > (v6 ? 128u : 32u) || c.list >= FB_MAX_BLACKLISTS) return false;
        const uint32_t bits = v6 ? 128u : 32u;
        const u128 all = v6 ? ~(u128)0 : (u128)0xFFFFFFFFu;
        const u128 hostmask = c.prefix == 0u ? all : (((u128)1 << (bits - c.prefix)) - 1u);
        const u128 a = v6 ? to128(c.addr) : (u128)c.addr[0];
        const u128 net = a & ~hostmask & all, bc = net | hostmask;  // IpNet::network() / broadcast()
        std::vector<Ev>& ev = v6 ? e6 : e4;
        ev.push_back(Ev{net, c.list, +1});
        if (bc != all) ev.push_back(Ev{bc + 1u, c.list, -1});
    }
    std::vector<u128> q4, q6;
    m4.clear();
    m6.clear();
    sweep(e4, q4, m4);
    sweep(e6, q6, m6);
    p4.resize(q4.size());
    for (size_t i = 0; i < q4.size(); ++i) p4[i] = (uint32_t)q4[i];
    p6.resize(q6.size());
    for (size_t i = 0; i < q6.size(); ++i)
        p6[i] = make_uint4((uint32_t)(q6[i] >> 96), (uint32_t)(q6[i] >> 64), (uint32_t)(q6[i] >> 32), (uint32_t)q6[i]);
    return true;
}

}  // namespace fbk
