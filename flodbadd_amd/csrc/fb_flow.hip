// fb_flow.hip -- gfx950 session (flow) table: upsert of SESSION records + integer counters.
//
// Replaces the per-packet DashMap upsert of process_parsed_packet (src/packets.rs:329-535):
// Entry::Occupied -> update_session_stats counters (src/packets.rs:111-120), Entry::Vacant ->
// new SessionInfo with the first packet's counters (src/packets.rs:383-391), and the
// PACKET_STATS new/updated counters (src/packets.rs:334-347).
//
// Table: open addressing, linear probing, 128-B slots (one line: tag + key + 6 u64 counters).
// The reference hashes Session with SipHash under a random per-process key (dashmap 6.1.0
// RandomState), so no hash value is a parity target; this table uses fb_flow_hash (below),
// a deterministic 64-bit mix of the 40-B session_key, identical on host and device.
// Cross-workgroup visibility (MI355X_MICROARCH.md "Valid forms"): every shared word is read
// and written with agent-scope atomics (sc1), key words are drained (vmcnt(0)) before the tag
// that publishes them; counters are device-scope atomic adds (order-independent integer sums,
// so results are bit-exact whatever the interleaving).
#include "fb_internal.h"

namespace fbk {

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

__device__ __forceinline__ unsigned long long ald(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Find-or-insert `key` (10 words).  Returns the slot or nullptr (table full / spin expired).
__device__ __forceinline__ FlowSlot* upsert(FlowSlot* table, unsigned long long mask,
                                            const uint32_t key[10], bool& inserted, uint32_t* err) {
    const unsigned long long h = flow_hash_words(key);
    const unsigned long long want = h | 2ull;  // 0 = empty, 1 = being inserted
    const unsigned long long kw0 = (unsigned long long)key[0] | ((unsigned long long)key[1] << 32);
    const unsigned long long kw1 = (unsigned long long)key[2] | ((unsigned long long)key[3] << 32);
    const unsigned long long kw2 = (unsigned long long)key[4] | ((unsigned long long)key[5] << 32);
    const unsigned long long kw3 = (unsigned long long)key[6] | ((unsigned long long)key[7] << 32);
    const unsigned long long kw4 = (unsigned long long)key[8] | ((unsigned long long)key[9] << 32);
    unsigned long long idx = h & mask;
    inserted = false;
    for (unsigned long long probe = 0; probe <= mask; ++probe) {
        FlowSlot* s = table + idx;
        unsigned long long* kp = reinterpret_cast<unsigned long long*>(s->key);
        unsigned long long t = ald(&s->tag);
        if (t == 0ull) {
            const unsigned long long old = atomicCAS(&s->tag, 0ull, 1ull);
            if (old == 0ull) {
                ast(kp + 0, kw0);
                ast(kp + 1, kw1);
                ast(kp + 2, kw2);
                ast(kp + 3, kw3);
                ast(kp + 4, kw4);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                ast(&s->tag, want);
                inserted = true;
                return s;
            }
            t = old;
        }
        uint32_t spins = 0u;
        while (t == 1ull) {  // another lane is publishing this slot's key
            __builtin_amdgcn_s_sleep(1);
            t = ald(&s->tag);
            if (++spins > (1u << 24)) { atomicOr(err, 2u); return nullptr; }
        }
        if (t == want && ald(kp + 0) == kw0 && ald(kp + 1) == kw1 && ald(kp + 2) == kw2 &&
            ald(kp + 3) == kw3 && ald(kp + 4) == kw4)
            return s;
        idx = (idx + 1ull) & mask;
    }
    atomicOr(err, 4u);  // table full
    return nullptr;
}

__device__ __forceinline__ void count_packet(FlowSlot* s, uint32_t plen, uint32_t iplen, bool orig) {
    // originator -> outbound_bytes/orig_pkts/orig_ip_bytes, else inbound/resp (packets.rs:111-120)
    atomicAdd(&s->cnt[orig ? 0 : 1], (unsigned long long)plen);
    atomicAdd(&s->cnt[orig ? 2 : 3], 1ull);
    atomicAdd(&s->cnt[orig ? 4 : 5], (unsigned long long)iplen);
}

__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0u) sh[wave] = v;
    __syncthreads();
    unsigned long long t = 0ull;
    for (uint32_t w = 0; w < blockDim.x / 64u; ++w) t += sh[w];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(256) void k_flow_update(const FlowParams P) {
    __shared__ unsigned long long sh[4];
    const unsigned long long n = P.stats->n_session;  // written by the parse kernel
    const uint32_t lim = (uint32_t)min(n, (unsigned long long)P.max_recs);
    unsigned long long n_new = 0ull, n_upd = 0ull;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += gridDim.x * blockDim.x) {
        const uint32_t* r = reinterpret_cast<const uint32_t*>(P.recs + i);
        const uint4 a = *reinterpret_cast<const uint4*>(r);
        const uint4 b = *reinterpret_cast<const uint4*>(r + 4);
        const uint2 c = *reinterpret_cast<const uint2*>(r + 8);
        const uint2 d = *reinterpret_cast<const uint2*>(r + 10);
        const uint32_t m = r[12];
        const uint32_t key[10] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y};
        bool ins;
        FlowSlot* s = upsert(P.table, P.mask, key, ins, P.error);
        if (s) {
            count_packet(s, d.x, d.y, (m >> 8) & FB_META_ORIGINATOR);
            n_new += ins;
            n_upd += !ins;
        }
    }
    n_new = block_sum(n_new, sh);
    n_upd = block_sum(n_upd, sh);
    if (threadIdx.x == 0) {
        P.partials[2 * blockIdx.x] = n_new;
        P.partials[2 * blockIdx.x + 1] = n_upd;
    }
}

__global__ __launch_bounds__(256) void k_flow_finish(fb_batch_stats* S, const unsigned long long* part,
                                                     uint32_t nblk, const uint32_t* err) {
    __shared__ unsigned long long sh[4];
    unsigned long long a = 0ull, b = 0ull;
    for (uint32_t i = threadIdx.x; i < nblk; i += blockDim.x) {
        a += part[2 * i];
        b += part[2 * i + 1];
    }
    a = block_sum(a, sh);
    b = block_sum(b, sh);
    if (threadIdx.x == 0) {
        S->new_sessions += a;
        S->updated_sessions += b;
        S->error |= *err;
    }
}

__global__ __launch_bounds__(256) void k_flow_export(const FlowSlot* T, unsigned long long cap,
                                                     fb_flow_rec* out, unsigned long long out_cap,
                                                     unsigned long long* d_n) {
    __shared__ unsigned long long sh[4];
    __shared__ unsigned long long s_base;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < cap; base += stride) {
        const unsigned long long i = base + threadIdx.x;
        const bool occ = i < cap && T[i].tag >= 2ull;
        const unsigned long long m = __ballot(occ);
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
        if (occ && pos < out_cap) {
            fb_flow_rec r;
            __builtin_memcpy(&r.key, T[i].key, 40);
            r.outbound_bytes = T[i].cnt[0];
            r.inbound_bytes = T[i].cnt[1];
            r.orig_pkts = T[i].cnt[2];
            r.resp_pkts = T[i].cnt[3];
            r.orig_ip_bytes = T[i].cnt[4];
            r.resp_ip_bytes = T[i].cnt[5];
            out[pos] = r;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_flow_count(const FlowSlot* T, unsigned long long cap,
                                                    unsigned long long* d_n) {
    __shared__ unsigned long long sh[4];
    unsigned long long c = 0ull;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride)
        c += T[i].tag >= 2ull;
    c = block_sum(c, sh);
    if (threadIdx.x == 0 && c) atomicAdd(d_n, c);
}

hipError_t launch_flow_update(const FlowParams& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(k_flow_update, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_flow_finish(fb_batch_stats* stats, const unsigned long long* partials, uint32_t nblk,
                              uint32_t* error, hipStream_t s) {
    hipLaunchKernelGGL(k_flow_finish, dim3(1), dim3(256), 0, s, stats, partials, nblk, error);
    return hipGetLastError();
}
hipError_t launch_flow_export(const FlowSlot* table, unsigned long long cap, fb_flow_rec* out,
                              unsigned long long out_cap, unsigned long long* d_n, hipStream_t s) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > 1024ull) g = 1024ull;
    if (g == 0ull) g = 1ull;
    hipLaunchKernelGGL(k_flow_export, dim3((uint32_t)g), dim3(256), 0, s, table, cap, out, out_cap, d_n);
    return hipGetLastError();
}
hipError_t launch_flow_count(const FlowSlot* table, unsigned long long cap, unsigned long long* d_n,
                             hipStream_t s) {
    unsigned long long g = (cap + 255ull) / 256ull;
    if (g > 1024ull) g = 1024ull;
    if (g == 0ull) g = 1ull;
    hipLaunchKernelGGL(k_flow_count, dim3((uint32_t)g), dim3(256), 0, s, table, cap, d_n);
    return hipGetLastError();
}

}  // namespace fbk

extern "C" uint64_t fb_flow_hash(const fb_session_key* key) {
    uint32_t w[10];
    __builtin_memcpy(w, key, 40);
    return fbk::flow_hash_words(w);
}
