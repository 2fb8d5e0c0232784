// parse_experiments.hip -- kernel variants that were measured and NOT adopted (tooling only;
// included by tools/ubench_parse.hip after flodbadd_amd/csrc/fb_parse.hip).
//
// Measured on MI355X (C2, 1M x 64 B, 8 rotating batches; k_parse_block = 44.6-45.2 us):
//   k_parse_pipe  71 us   frame waves + control wave, loop-carried prefetch of round k+1; its DNS
//                         registers were indexed by a runtime slot (scratch) and every round waited
//                         for its own store completions.
//   k_parse_ctl   51 us   control wave, two LDS slots, look-back of k-1 beside the loads of k.
//   k_parse_ctl1  47.7 us control wave, one slot, loads of k issued before waiting for k-1's prefix.
//   k_parse_2p    67.6 us two passes per block chunk (count, one look-back, re-read + store).
//   first-round stagger of k_parse_block (b * 10..60 ns): monotonically slower (+1.8..+20 us).
// Common cause (per-unit stamps): inside a round every block's loads are served interleaved with
// all others, so nearly every unit's look-back waits for the round's slowest predecessor.
namespace fbk {
// ============================================================================================
// Block-level pipeline with a control wave (the product kernel).
//
// A block = kExpFrameWaves frame waves + 1 control wave.  A unit = one block-round =
// kExpFrameWaves x U wave-tiles x 64 frames; block b (of G co-resident blocks) owns units
// b, b+G, ...; inside a unit frame wave w owns frames [w*U*64, (w+1)*U*64), so packet order =
// (wave, tile, lane).  Round k of a block (unit u_k):
//   frame waves: wait headers(u_k) -> classify -> stage records in LDS slot k%2, counts
//                -> issue header loads of u_{k+1}, offset loads of u_{k+2}           | B(k)
//                -> store u_{k-1}'s records from slot (k-1)%2 with its prefix       | loop
//   control    : | B(k) -> publish AGG(u_k), look-back(u_k) -> prefix -> INC(u_k)   | loop
// B(k) hands the control wave round k's counts and the frame waves round k-1's prefix.  The
// look-back of u_k therefore overlaps the frame waves' stores of u_{k-1}, their wait for u_{k+1}'s
// headers and their classification of u_{k+1}: HBM sees loads, stores and the look-back hop at
// once.  The control wave issues no frame loads, so its polls never queue behind them.
// ============================================================================================
template <int U, uint32_t FLAGS>
__global__ __launch_bounds__(kThreads) void k_parse_pipe(const ParseParams P) {
    constexpr uint32_t kFW = kExpFrameWaves;
    constexpr uint32_t WF = 64u * U;     // frames per frame wave per unit
    constexpr uint32_t UF = WF * kFW;    // frames per unit
    static_assert(kThreads == 64 * (kExpFrameWaves + 1), "build with -DFB_BLOCK_THREADS=64*(FB_FRAME_WAVES+1)");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const bool control = wave == kFW;
    const uint32_t G = gridDim.x, T = P.num_tiles;  // T = units
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;

    __shared__ DevConfig s_cfg;                                     // service bitmap + tables
    __shared__ unsigned long long s_stage_all[kFW][2][WF * 7];     // per frame wave, 2 slots
    __shared__ uint32_t s_cnt[2][kFW][4];                          // sessions, dns, filtered|tcp, v4|bad
    __shared__ unsigned long long s_excl[2];

    uint32_t u = blockIdx.x;  // G <= T: every block owns at least one unit
    uint2 o[U], on[U];
    Hdr h[U];
    auto load_off = [&](uint32_t unit, uint2 (&dst)[U]) {
        const uint32_t f0 = unit * UF + wave * WF;
#pragma unroll
        for (int r = 0; r < U; ++r) {
            const uint32_t i = f0 + r * 64u + lane;
            dst[r] = make_uint2(P.offsets[min(i, P.n)], P.offsets[min(i + 1u, P.n)]);  // n+1 entries
        }
    };
    if (!control) {
        load_off(u, o);
#pragma unroll
        for (int r = 0; r < U; ++r) load_headers1(rs, o[r].x, h[r]);
        load_off(min(u + G, T - 1u), on);
    }
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
    uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;  // pre-filter counters (control wave)
    unsigned long long m_dns[2][U];                     // DNS masks + records of rounds k, k-1
    uint4 dnsw[2][U];
    uint32_t cs_prev = 0u;
    bool have_prev = false;
    uint32_t slot = 0u;
    for (;;) {
        const bool cur = u < T;
        if (!control) {
            if (cur) {
                // ---- classify u, stage in slot `slot` -------------------------------------------
                const uint32_t f0 = u * UF + wave * WF;
                unsigned long long* st = s_stage_all[wave][slot];
                uint32_t cs = 0u, cd = 0u, wf = 0u, wt = 0u, w4 = 0u, wb = 0u;
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint32_t i = f0 + r * 64u + lane;
                    const bool valid = i < P.n;
                    Pkt k;
                    process_frame(rs, cfg, cfg->service_bitmap, h[r], valid ? o[r].x : 1u, valid ? o[r].y : 0u,
                                  P.frames_bytes, i, k);
                    const bool is_s = valid && k.cls == FB_CLASS_SESSION;
                    const bool is_d = valid && k.cls == FB_CLASS_DNS;
                    const bool is_f = valid && k.cls == FB_CLASS_FILTERED;
                    const bool counted = is_s || is_f;
                    const unsigned long long m_sess = __ballot(is_s);
                    m_dns[slot][r] = __ballot(is_d);
                    dnsw[slot][r] = make_uint4(k.w[0], k.w[1], k.w[2], k.w[3]);
                    if (is_s) {
                        unsigned long long* d = st + (size_t)(cs + __popcll(m_sess & lmask)) * 7;
#pragma unroll
                        for (int w = 0; w < 7; ++w)
                            d[w] = (unsigned long long)k.w[2 * w] | ((unsigned long long)k.w[2 * w + 1] << 32);
                    }
                    cs += (uint32_t)__popcll(m_sess);
                    cd += (uint32_t)__popcll(m_dns[slot][r]);
                    wf += __popcll(__ballot(is_f));
                    wt += __popcll(__ballot(counted && k.tcp));
                    w4 += __popcll(__ballot(counted && k.v4));
                    wb += __popcll(__ballot(valid && k.bad));
                    if (valid && P.cls) P.cls[i] = (uint8_t)k.cls;
                }
                if (lane == 0u) {
                    s_cnt[slot][wave][0] = cs;
                    s_cnt[slot][wave][1] = cd;
                    s_cnt[slot][wave][2] = wf | (wt << 16);
                    s_cnt[slot][wave][3] = w4 | (wb << 16);
                }
                // ---- prefetch: headers of the next unit, offsets of the one after ------------------
                if (u + G < T) {
#pragma unroll
                    for (int r = 0; r < U; ++r) o[r] = on[r];
#pragma unroll
                    for (int r = 0; r < U; ++r) load_headers1(rs, o[r].x, h[r]);
                    load_off(min(u + 2u * G, T - 1u), on);
                }
                cs_prev = cs;  // used after B(k) for round k's stores (next iteration)
            }
        }
        __syncthreads();  // B(k): round k's counts; round k-1's prefix (control, previous iteration)
        if (control) {
            if (cur) {
                uint32_t bs = 0u, bd = 0u;
#pragma unroll
                for (uint32_t w = 0; w < kFW; ++w) {
                    bs += s_cnt[slot][w][0];
                    bd += s_cnt[slot][w][1];
                    a_f += s_cnt[slot][w][2] & 0xFFFFu;
                    a_t += s_cnt[slot][w][2] >> 16;
                    a_4 += s_cnt[slot][w][3] & 0xFFFFu;
                    a_b += s_cnt[slot][w][3] >> 16;
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
                if (lane == 0u) s_excl[slot] = excl;
                if (u == T - 1u && P.stats && !(FLAGS & kNoLookback)) {
                    // the last unit's owner: own counters first (this is the block's last unit)
                    if (lane == 0u) {
                        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
                        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
                    }
                    write_batch_stats(P, excl + agg, G);
                }
            }
        } else if (have_prev && !(FLAGS & kNoStore)) {
            // ---- stores of round k-1 (slot ^ 1), whose prefix the control wave wrote before B(k) --
            const uint32_t ps = slot ^ 1u;
            const unsigned long long bex = s_excl[ps];
            uint32_t base_s = (uint32_t)(bex & ((1ull << 28) - 1ull));
            uint32_t base_d = (uint32_t)(bex >> 28);
            for (uint32_t w = 0; w < wave; ++w) {
                base_s += s_cnt[ps][w][0];
                base_d += s_cnt[ps][w][1];
            }
            const uint32_t cs = s_cnt[ps][wave][0];
            const unsigned long long* st = s_stage_all[wave][ps];
            if (P.out && cs) {
                // [base_s*56, (base_s+cs)*56) is 8-B aligned: 16-B aligned body + 8-B head/tail
                unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7;
                const uint32_t units = cs * 7, head = base_s & 1u, body = (units - head) >> 1;
                if (head && lane == 0u) g8[0] = st[0];
                uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                for (uint32_t c = lane; c < body; c += 64u) {
                    const unsigned long long x = st[head + 2 * c], y = st[head + 2 * c + 1];
                    g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                }
                if (lane == 0u && head + 2 * body < units) g8[units - 1] = st[units - 1];
            }
            if (P.dns) {
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    if ((m_dns[ps][r] >> lane) & 1ull) {
                        fb_dns_out d;
                        d.pkt_index = dnsw[ps][r].x;
                        d.payload_offset = dnsw[ps][r].y;
                        d.payload_length = dnsw[ps][r].z;
                        d.protocol = (uint8_t)(dnsw[ps][r].w & 0xffu);
                        d.family = (uint8_t)(dnsw[ps][r].w >> 8);
                        d.reserved = 0;
                        P.dns[base_d + __popcll(m_dns[ps][r] & lmask)] = d;
                    }
                    base_d += (uint32_t)__popcll(m_dns[ps][r]);
                }
            }
        }
        if (!cur) break;
        have_prev = true;
        u += G;
        slot ^= 1u;
    }
    (void)cs_prev;
    // every block publishes its pre-filter counters (the last unit's owner did so above)
    const bool owner_last = T > 0u && (T - 1u) % G == blockIdx.x;
    if (control && !owner_last && lane == 0u && !(FLAGS & kNoLookback)) {
        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
    }
}


// ============================================================================================
// k_parse_ctl: the block-round kernel with the look-back moved off the critical path.
//
// A block = kCtlFW frame waves + 1 control wave; unit = kCtlFW x U wave-tiles x 64 frames.
// Step k (unit u_k in LDS slot k%2; the loop is unrolled by two so slots and the DNS registers
// are compile-time indexed -- a runtime-indexed register array would live in scratch):
//   frame waves: loads(u_k) -> classify -> stage records in slot k%2, counts       | B1
//                -> store u_{k-1} from slot (k-1)%2 with its prefix                  | B2
//   control    : look-back(u_{k-1}) -> prefix, INC(u_{k-1})                          | B1
//                -> publish AGG(u_k)                                                 | B2
// The look-back of u_{k-1} runs while the frame waves wait for u_k's header loads; nothing is
// prefetched across a loop iteration, so no wait ever covers a younger load than it needs.
// ============================================================================================
template <int U, uint32_t FLAGS, bool PARSED = false>
__global__ __launch_bounds__(kCtlThreads) void k_parse_ctl(const ParseParams P) {
    constexpr uint32_t kFW = kCtlFW;
    constexpr uint32_t WF = 64u * U;     // frames per frame wave per unit
    constexpr uint32_t UF = WF * kFW;    // frames per unit
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const bool control = wave == kFW;
    const uint32_t G = gridDim.x, T = P.num_tiles;  // T = units
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;

    __shared__ DevConfig s_cfg;
    __shared__ unsigned long long s_rec[kFW][2][WF * 7];  // per frame wave, 2 slots of records
    __shared__ uint32_t s_cnt[2][kFW][4];                 // sessions, dns, filtered|tcp, v4|bad
    __shared__ unsigned long long s_excl[2];
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        uint4* dst = reinterpret_cast<uint4*>(&s_cfg);
        for (uint32_t q = tid; q < sizeof(DevConfig) / 16; q += kCtlThreads) dst[q] = src[q];
        // Zero the other parity's error word for the next launch (the previous launch, which
        // used it, has completed: launches on one context are stream-ordered).
        if (blockIdx.x == 0u && tid == 0u) *P.error_next = 0u;
    }
    __syncthreads();
    const DevConfig* cfg = &s_cfg;

    const unsigned long long lmask = (1ull << lane) - 1ull;
    uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;  // pre-filter counters (control wave)
    unsigned long long m_dns[2][U];                     // DNS masks + records per slot (frame waves)
    uint4 dnsw[2][U];
    uint32_t u = blockIdx.x, prev = 0u;
    bool have_prev = false, done = false;

    auto step = [&](auto par) {
        constexpr int S = decltype(par)::value;
        const bool cur = u < T;
        if (!control) {
            if (cur) {
                const uint32_t f0 = u * UF + wave * WF;
                uint2 o[U];
                Hdr h[U];
                uint4 pin[U][4];
                if constexpr (!PARSED) {
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        const uint32_t i = f0 + r * 64u + lane;
                        o[r] = make_uint2(P.offsets[min(i, P.n)], P.offsets[min(i + 1u, P.n)]);
                    }
#pragma unroll
                    for (int r = 0; r < U; ++r) load_headers1(rs, o[r].x, h[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        const uint32_t i = min(f0 + r * 64u + lane, P.n - 1u);
                        const uint4* q = reinterpret_cast<const uint4*>(P.parsed + i);
                        pin[r][0] = q[0];
                        pin[r][1] = q[1];
                        pin[r][2] = q[2];
                        const uint2 t2 = *reinterpret_cast<const uint2*>(q + 3);
                        pin[r][3] = make_uint4(t2.x, t2.y, 0u, 0u);
                    }
                }
                unsigned long long* st = s_rec[wave][S];
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
                        const uint4 a = pin[r][0], b = pin[r][1], c = pin[r][2], d = pin[r][3];
                        const uint32_t srcw[4] = {a.x, a.y, a.z, a.w}, dstw[4] = {b.x, b.y, b.z, b.w};
                        const uint32_t proto = c.y & 0xffu, fam = (c.y >> 8) & 0xffu;
                        k.bad = false;
                        k.cls = FB_CLASS_DROP;
                        k.tcp = k.v4 = false;
                        if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                            classify_session(cfg, cfg->service_bitmap, proto, fam, srcw, dstw, c.x & 0xffffu,
                                             c.x >> 16, (d.x >> 8) & 1u, d.x & 0xffu, c.z, c.w, d.y, k);
                    }
                    const bool is_s = valid && k.cls == FB_CLASS_SESSION;
                    const bool is_d = valid && k.cls == FB_CLASS_DNS;
                    const bool is_f = valid && k.cls == FB_CLASS_FILTERED;
                    const bool counted = is_s || is_f;
                    const unsigned long long m_sess = __ballot(is_s);
                    m_dns[S][r] = __ballot(is_d);
                    dnsw[S][r] = make_uint4(k.w[0], k.w[1], k.w[2], k.w[3]);
                    if (is_s) {
                        unsigned long long* d = st + (size_t)(cs + __popcll(m_sess & lmask)) * 7;
#pragma unroll
                        for (int w = 0; w < 7; ++w)
                            d[w] = (unsigned long long)k.w[2 * w] | ((unsigned long long)k.w[2 * w + 1] << 32);
                    }
                    cs += (uint32_t)__popcll(m_sess);
                    cd += (uint32_t)__popcll(m_dns[S][r]);
                    wf += __popcll(__ballot(is_f));
                    wt += __popcll(__ballot(counted && k.tcp));
                    w4 += __popcll(__ballot(counted && k.v4));
                    wb += __popcll(__ballot(valid && k.bad));
                    if (valid && P.cls) P.cls[i] = (uint8_t)k.cls;
                }
                if (lane == 0u) {
                    s_cnt[S][wave][0] = cs;
                    s_cnt[S][wave][1] = cd;
                    s_cnt[S][wave][2] = wf | (wt << 16);
                    s_cnt[S][wave][3] = w4 | (wb << 16);
                }
            }
        } else if (have_prev) {
            // ---- look-back of the previous unit (slot S^1), overlapping the frame loads ---------
            uint32_t bs = 0u, bd = 0u;
#pragma unroll
            for (uint32_t w = 0; w < kFW; ++w) {
                bs += s_cnt[S ^ 1][w][0];
                bd += s_cnt[S ^ 1][w][1];
            }
            const unsigned long long agg = (unsigned long long)bs | ((unsigned long long)bd << 28);
            unsigned long long excl;
            if (FLAGS & kNoLookback) {
                excl = (unsigned long long)prev * UF;
            } else {
                uint32_t spins;
                excl = lookback_unit<FLAGS>(P, prev, spins);
                if (lane == 0u) ast(P.tagg + prev, st_pack(ep, true, excl + agg));
                if constexpr ((FLAGS & kStamps) != 0u)
                    if (lane == 0u) {
                        P.dbg[4ull * prev + 2] = __builtin_amdgcn_s_memrealtime();
                        P.dbg[4ull * prev + 3] = spins;
                    }
            }
            if (lane == 0u) s_excl[S ^ 1] = excl;
            if (prev == T - 1u && P.stats && !(FLAGS & kNoLookback)) {
                // the last unit's owner: own counters first (this is the block's last unit)
                if (lane == 0u) {
                    ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
                    ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
                }
                write_batch_stats(P, excl + agg, G);
            }
        }
        __syncthreads();  // B1: unit u's counts and records; prev's prefix
        if (!control) {
            if (have_prev && !(FLAGS & kNoStore)) {
                const unsigned long long bex = s_excl[S ^ 1];
                uint32_t base_s = (uint32_t)(bex & ((1ull << 28) - 1ull));
                uint32_t base_d = (uint32_t)(bex >> 28);
                for (uint32_t w = 0; w < wave; ++w) {
                    base_s += s_cnt[S ^ 1][w][0];
                    base_d += s_cnt[S ^ 1][w][1];
                }
                const uint32_t cs = s_cnt[S ^ 1][wave][0];
                const unsigned long long* st = s_rec[wave][S ^ 1];
                if (P.out && cs) {
                    // [base_s*56, (base_s+cs)*56) is 8-B aligned: 16-B aligned body + 8-B head/tail
                    unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7;
                    const uint32_t units = cs * 7, head = base_s & 1u, body = (units - head) >> 1;
                    if (head && lane == 0u) g8[0] = st[0];
                    uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                    for (uint32_t c = lane; c < body; c += 64u) {
                        const unsigned long long x = st[head + 2 * c], y = st[head + 2 * c + 1];
                        g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                    }
                    if (lane == 0u && head + 2 * body < units) g8[units - 1] = st[units - 1];
                }
                if (P.dns) {
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        if ((m_dns[S ^ 1][r] >> lane) & 1ull) {
                            const uint4 dw = dnsw[S ^ 1][r];
                            fb_dns_out d;
                            d.pkt_index = dw.x;
                            d.payload_offset = dw.y;
                            d.payload_length = dw.z;
                            d.protocol = (uint8_t)(dw.w & 0xffu);
                            d.family = (uint8_t)(dw.w >> 8);
                            d.reserved = 0;
                            P.dns[base_d + __popcll(m_dns[S ^ 1][r] & lmask)] = d;
                        }
                        base_d += (uint32_t)__popcll(m_dns[S ^ 1][r]);
                    }
                }
            }
        } else if (cur) {
            // ---- publish unit u's aggregate (its look-back runs in the next step) --------------
            uint32_t bs = 0u, bd = 0u;
#pragma unroll
            for (uint32_t w = 0; w < kFW; ++w) {
                bs += s_cnt[S][w][0];
                bd += s_cnt[S][w][1];
                a_f += s_cnt[S][w][2] & 0xFFFFu;
                a_t += s_cnt[S][w][2] >> 16;
                a_4 += s_cnt[S][w][3] & 0xFFFFu;
                a_b += s_cnt[S][w][3] >> 16;
            }
            if constexpr ((FLAGS & kStamps) != 0u)
                if (lane == 0u) P.dbg[4ull * u] = __builtin_amdgcn_s_memrealtime();
            if (lane == 0u && !(FLAGS & kNoLookback))
                ast(P.tagg + u, st_pack(ep, false, (unsigned long long)bs | ((unsigned long long)bd << 28)));
        }
        __syncthreads();  // B2: slot S^1 stored; s_cnt/s_excl reuse
        if (!cur) {
            done = true;
        } else {
            have_prev = true;
            prev = u;
            u += G;
        }
    };
    while (!done) {
        step(IC<0>{});
        if (done) break;
        step(IC<1>{});
    }
    // every block publishes its pre-filter counters (the last unit's owner did so above)
    const bool owner_last = T > 0u && (T - 1u) % G == blockIdx.x;
    if (control && !owner_last && lane == 0u && !(FLAGS & kNoLookback)) {
        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
    }
}

// ============================================================================================
// k_parse_ctl1: control wave + ONE record slot; the frame waves issue unit k's header loads
// before they wait for unit k-1's prefix, so the look-back overlaps the loads:
//   frame waves: loads(u_k) | B0 | store(u_{k-1}) from the slot; classify(u_k); stage in slot | B1
//   control    :            | B0 |                                                        | B1
//                -> publish AGG(u_k), look-back(u_k) -> prefix      (runs into the next step)
// ============================================================================================
template <int U, uint32_t FLAGS, bool PARSED = false, int NW = 8>
__global__ __launch_bounds__(kCtlThreads) void k_parse_ctl1(const ParseParams P) {
    constexpr uint32_t kFW = kCtlFW;
    constexpr uint32_t WF = 64u * U;     // frames per frame wave per unit
    constexpr uint32_t UF = WF * kFW;    // frames per unit
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const bool control = wave == kFW;
    const uint32_t G = gridDim.x, T = P.num_tiles;  // T = units
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;

    __shared__ DevConfig s_cfg;
    __shared__ unsigned long long s_rec[kFW][WF * 7];  // per frame wave: the staged unit's records
    __shared__ uint4 s_dns[kFW][WF];                   // ... and its DNS records (compacted)
    __shared__ uint32_t s_cnt[kFW][4];                 // sessions, dns, filtered|tcp, v4|bad
    __shared__ unsigned long long s_excl;
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        uint4* dst = reinterpret_cast<uint4*>(&s_cfg);
        for (uint32_t q = tid; q < sizeof(DevConfig) / 16; q += kCtlThreads) dst[q] = src[q];
        if (blockIdx.x == 0u && tid == 0u) *P.error_next = 0u;  // next launch's error word
    }
    __syncthreads();
    const DevConfig* cfg = &s_cfg;

    const unsigned long long lmask = (1ull << lane) - 1ull;
    uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;  // pre-filter counters (control wave)
    uint32_t u = blockIdx.x, prev = 0u;
    bool have_prev = false;
    for (;;) {
        const bool cur = u < T;
        uint2 o[U];
        Hdr h[U];
        uint4 pin[U][4];
        if (!control && cur) {
            const uint32_t f0 = u * UF + wave * WF;
            if constexpr (!PARSED) {
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint32_t i = f0 + r * 64u + lane;
                    o[r] = make_uint2(P.offsets[min(i, P.n)], P.offsets[min(i + 1u, P.n)]);
                }
#pragma unroll
                for (int r = 0; r < U; ++r) load_headers1(rs, o[r].x, h[r]);
            } else {
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint32_t i = min(f0 + r * 64u + lane, P.n - 1u);
                    const uint4* q = reinterpret_cast<const uint4*>(P.parsed + i);
                    pin[r][0] = q[0];
                    pin[r][1] = q[1];
                    pin[r][2] = q[2];
                    const uint2 t2 = *reinterpret_cast<const uint2*>(q + 3);
                    pin[r][3] = make_uint4(t2.x, t2.y, 0u, 0u);
                }
            }
        }
        __syncthreads();  // B0: prev's prefix (control, previous iteration)
        if (!control) {
            // ---- stores of prev (the staged unit) while u's loads are in flight -------------------
            if (have_prev && !(FLAGS & kNoStore)) {
                const unsigned long long bex = s_excl;
                uint32_t base_s = (uint32_t)(bex & ((1ull << 28) - 1ull));
                uint32_t base_d = (uint32_t)(bex >> 28);
                for (uint32_t w = 0; w < wave; ++w) {
                    base_s += s_cnt[w][0];
                    base_d += s_cnt[w][1];
                }
                const uint32_t cs = s_cnt[wave][0];
                const unsigned long long* st = s_rec[wave];
                if (P.out && cs) {
                    // [base_s*56, (base_s+cs)*56) is 8-B aligned: 16-B aligned body + 8-B head/tail
                    unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7;
                    const uint32_t units = cs * 7, head = base_s & 1u, body = (units - head) >> 1;
                    if (head && lane == 0u) g8[0] = st[0];
                    uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                    for (uint32_t c = lane; c < body; c += 64u) {
                        const unsigned long long x = st[head + 2 * c], y = st[head + 2 * c + 1];
                        g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                    }
                    if (lane == 0u && head + 2 * body < units) g8[units - 1] = st[units - 1];
                }
                const uint32_t cd = s_cnt[wave][1];
                if (P.dns && cd) {
                    for (uint32_t c = lane; c < cd; c += 64u) {
                        const uint4 dw = s_dns[wave][c];
                        fb_dns_out d;
                        d.pkt_index = dw.x;
                        d.payload_offset = dw.y;
                        d.payload_length = dw.z;
                        d.protocol = (uint8_t)(dw.w & 0xffu);
                        d.family = (uint8_t)(dw.w >> 8);
                        d.reserved = 0;
                        P.dns[base_d + c] = d;
                    }
                }
            }
            // ---- classify u, stage in the slot (the stores above read it first: same wave) -------
            if (cur) {
                const uint32_t f0 = u * UF + wave * WF;
                unsigned long long* st = s_rec[wave];
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
                        const uint4 a = pin[r][0], b = pin[r][1], c = pin[r][2], d = pin[r][3];
                        const uint32_t srcw[4] = {a.x, a.y, a.z, a.w}, dstw[4] = {b.x, b.y, b.z, b.w};
                        const uint32_t proto = c.y & 0xffu, fam = (c.y >> 8) & 0xffu;
                        k.bad = false;
                        k.cls = FB_CLASS_DROP;
                        k.tcp = k.v4 = false;
                        if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                            classify_session(cfg, cfg->service_bitmap, proto, fam, srcw, dstw, c.x & 0xffffu,
                                             c.x >> 16, (d.x >> 8) & 1u, d.x & 0xffu, c.z, c.w, d.y, k);
                    }
                    const bool is_s = valid && k.cls == FB_CLASS_SESSION;
                    const bool is_d = valid && k.cls == FB_CLASS_DNS;
                    const bool is_f = valid && k.cls == FB_CLASS_FILTERED;
                    const bool counted = is_s || is_f;
                    const unsigned long long m_sess = __ballot(is_s);
                    const unsigned long long m_dn = __ballot(is_d);
                    if (is_d) s_dns[wave][cd + __popcll(m_dn & lmask)] = make_uint4(k.w[0], k.w[1], k.w[2], k.w[3]);
                    if (is_s) {
                        unsigned long long* d = st + (size_t)(cs + __popcll(m_sess & lmask)) * 7;
#pragma unroll
                        for (int w = 0; w < 7; ++w)
                            d[w] = (unsigned long long)k.w[2 * w] | ((unsigned long long)k.w[2 * w + 1] << 32);
                    }
                    cs += (uint32_t)__popcll(m_sess);
                    cd += (uint32_t)__popcll(m_dn);
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
            }
        }
        __syncthreads();  // B1: u's counts and records staged; prev stored
        if (!cur) break;
        if (control) {
            // ---- publish AGG(u) and look back; overlaps the next iteration's loads ---------------
            uint32_t bs = 0u, bd = 0u;
#pragma unroll
            for (uint32_t w = 0; w < kFW; ++w) {
                bs += s_cnt[w][0];
                bd += s_cnt[w][1];
                a_f += s_cnt[w][2] & 0xFFFFu;
                a_t += s_cnt[w][2] >> 16;
                a_4 += s_cnt[w][3] & 0xFFFFu;
                a_b += s_cnt[w][3] >> 16;
            }
            const unsigned long long agg = (unsigned long long)bs | ((unsigned long long)bd << 28);
            unsigned long long excl;
            if (FLAGS & kNoLookback) {
                excl = (unsigned long long)u * UF;
            } else {
                if (lane == 0u) ast(P.tagg + u, st_pack(ep, false, agg));
                uint32_t spins;
                excl = lookback_unit<FLAGS, NW>(P, u, spins);
                if (lane == 0u) ast(P.tagg + u, st_pack(ep, true, excl + agg));
                if constexpr ((FLAGS & kStamps) != 0u)
                    if (lane == 0u) {
                        P.dbg[4ull * u + 2] = __builtin_amdgcn_s_memrealtime();
                        P.dbg[4ull * u + 3] = spins;
                    }
            }
            if (lane == 0u) s_excl = excl;
            if (u == T - 1u && P.stats && !(FLAGS & kNoLookback)) {
                if (lane == 0u) {
                    ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
                    ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
                }
                write_batch_stats(P, excl + agg, G);
            }
        }
        have_prev = true;
        prev = u;
        u += G;
    }
    (void)prev;
    const bool owner_last = T > 0u && (T - 1u) % G == blockIdx.x;
    if (control && !owner_last && lane == 0u && !(FLAGS & kNoLookback)) {
        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
    }
}

// ============================================================================================
// k_parse_2p: two passes per block-chunk, ONE look-back per chunk.
#ifndef FB_2P_MINW
#define FB_2P_MINW 4  // min waves per SIMD: 2 blocks of 512 lanes per CU
#endif
//
// A unit = one block-round = kWaves x U x 64 contiguous frames (wave w owns tiles
// [w*U, (w+1)*U) of the chunk, packet order = (wave, tile, lane)).  Per unit:
//   pass 1: every wave issues all its offset + header loads (U tiles in flight), decodes and
//           classifies for COUNTS only (nothing is kept), writes the class byte   | barrier
//   wave 0: publishes the unit's aggregate, one look-back over <= 64*NW predecessors per
//           round trip                                                          | barrier
//   pass 2: every wave re-reads its headers (the round's frames were just read: L2 / Infinity
//           Cache hits, not HBM), re-derives the records and writes them at their final
//           offsets (LDS-staged, coalesced 16-B stores) + DNS records.
// The look-back wait is paid once per round instead of once per small unit, and no record is
// held across it, so registers and LDS stay small.  Within a round every block is delayed by
// the round's slowest predecessor (its loads are served interleaved with everyone else's): that
// skew is the price of ordered compaction and is paid once per round here.
// ============================================================================================
template <int U, uint32_t FLAGS, bool PARSED = false, int NW = 8>
__global__ __launch_bounds__(kThreads, FB_2P_MINW) void k_parse_2p(const ParseParams P) {
    constexpr uint32_t kWaves = kThreads / 64;
    constexpr uint32_t WF = 64u * U;      // frames per wave per unit
    constexpr uint32_t UF = WF * kWaves;  // frames per unit
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t G = gridDim.x, T = P.num_tiles;  // T = units
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.frames, (short)0, (int)P.frames_bytes, 0x00020000);
    const uint32_t ep = P.epoch;

    __shared__ DevConfig s_cfg;
    __shared__ unsigned long long s_stage_all[kWaves][64 * 7];  // one tile of records per wave
    __shared__ uint32_t s_cnt[kWaves][4];                        // sessions, dns, filtered|tcp, v4|bad
    __shared__ unsigned long long s_excl;
    unsigned long long* s_stage = s_stage_all[wave];
    {
        const uint4* src = reinterpret_cast<const uint4*>(P.cfg);
        uint4* dst = reinterpret_cast<uint4*>(&s_cfg);
        for (uint32_t q = tid; q < sizeof(DevConfig) / 16; q += kThreads) dst[q] = src[q];
        if (blockIdx.x == 0u && tid == 0u) *P.error_next = 0u;  // next launch's error word
    }
    __syncthreads();
    const DevConfig* cfg = &s_cfg;
    const unsigned long long lmask = (1ull << lane) - 1ull;
    uint32_t a_f = 0u, a_t = 0u, a_4 = 0u, a_b = 0u;  // pre-filter counters (wave 0 keeps them)

    // decode + classify tile r of this wave in unit u (loads issued by the caller)
    auto classify = [&](uint32_t i, const Hdr& h, uint2 o, const uint4 (&pin)[4], Pkt& k) {
        const bool valid = i < P.n;
        if constexpr (!PARSED) {
            process_frame(rs, cfg, cfg->service_bitmap, h, valid ? o.x : 1u, valid ? o.y : 0u, P.frames_bytes, i, k);
        } else {
            const uint4 a = pin[0], b = pin[1], c = pin[2], d = pin[3];
            const uint32_t srcw[4] = {a.x, a.y, a.z, a.w}, dstw[4] = {b.x, b.y, b.z, b.w};
            const uint32_t proto = c.y & 0xffu, fam = (c.y >> 8) & 0xffu;
            k.bad = false;
            k.cls = FB_CLASS_DROP;
            k.tcp = k.v4 = false;
            if ((proto == 6u || proto == 17u) && (fam == 2u || fam == 10u))
                classify_session(cfg, cfg->service_bitmap, proto, fam, srcw, dstw, c.x & 0xffffu, c.x >> 16,
                                 (d.x >> 8) & 1u, d.x & 0xffu, c.z, c.w, d.y, k);
        }
        return valid;
    };
    auto load_unit = [&](uint32_t f0, uint2 (&o)[U], Hdr (&h)[U], uint4 (&pin)[U][4]) {
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
                const uint2 t2 = *reinterpret_cast<const uint2*>(q + 3);
                pin[r][3] = make_uint4(t2.x, t2.y, 0u, 0u);
            }
        }
    };

    for (uint32_t u = blockIdx.x; u < T; u += G) {
        const uint32_t f0 = u * UF + wave * WF;  // first frame of this wave
        // ---- pass 1: counts ------------------------------------------------------------------
        {
            uint2 o[U];
            Hdr h[U];
            uint4 pin[U][4];
            load_unit(f0, o, h, pin);
            uint32_t cs = 0u, cd = 0u, wf = 0u, wt = 0u, w4 = 0u, wb = 0u;
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = f0 + r * 64u + lane;
                Pkt k;
                const bool valid = classify(i, h[r], o[r], pin[r], k);
                const bool is_s = valid && k.cls == FB_CLASS_SESSION;
                const bool is_d = valid && k.cls == FB_CLASS_DNS;
                const bool is_f = valid && k.cls == FB_CLASS_FILTERED;
                const bool counted = is_s || is_f;
                cs += (uint32_t)__popcll(__ballot(is_s));
                cd += (uint32_t)__popcll(__ballot(is_d));
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
        }
        __syncthreads();  // counts of every wave
        // ---- publish + look-back (wave 0) -------------------------------------------------------
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
                excl = lookback_unit<FLAGS, NW>(P, u, spins);
                if (lane == 0u) ast(P.tagg + u, st_pack(ep, true, excl + agg));
                if constexpr ((FLAGS & kStamps) != 0u)
                    if (lane == 0u) {
                        P.dbg[4ull * u + 2] = __builtin_amdgcn_s_memrealtime();
                        P.dbg[4ull * u + 3] = spins;
                    }
            }
            if (lane == 0u) s_excl = excl;
            if (u == T - 1u && P.stats && !(FLAGS & kNoLookback)) {
                if (lane == 0u) {
                    ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
                    ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
                }
                write_batch_stats(P, excl + agg, G);
            }
        }
        __syncthreads();  // s_excl
        // ---- pass 2: records at their final offsets ----------------------------------------------
        if (!(FLAGS & kNoStore)) {
            const unsigned long long bex = s_excl;
            uint32_t base_s = (uint32_t)(bex & ((1ull << 28) - 1ull));
            uint32_t base_d = (uint32_t)(bex >> 28);
            for (uint32_t w = 0; w < wave; ++w) {
                base_s += s_cnt[w][0];
                base_d += s_cnt[w][1];
            }
            uint2 o[U];
            Hdr h[U];
            uint4 pin[U][4];
            load_unit(f0, o, h, pin);
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t i = f0 + r * 64u + lane;
                Pkt k;
                const bool valid = classify(i, h[r], o[r], pin[r], k);
                const bool is_s = valid && k.cls == FB_CLASS_SESSION;
                const bool is_d = valid && k.cls == FB_CLASS_DNS;
                const unsigned long long m_sess = __ballot(is_s);
                const unsigned long long m_dn = __ballot(is_d);
                const uint32_t ps = (uint32_t)__popcll(m_sess);
                if (P.out && ps) {
                    if (is_s) {
                        unsigned long long* d = s_stage + (size_t)__popcll(m_sess & lmask) * 7;
#pragma unroll
                        for (int w = 0; w < 7; ++w)
                            d[w] = (unsigned long long)k.w[2 * w] | ((unsigned long long)k.w[2 * w + 1] << 32);
                    }
                    // [base_s*56, (base_s+ps)*56) is 8-B aligned: 16-B aligned body + 8-B head/tail
                    unsigned long long* g8 = reinterpret_cast<unsigned long long*>(P.out) + (size_t)base_s * 7;
                    const uint32_t units = ps * 7, head = base_s & 1u, body = (units - head) >> 1;
                    if (head && lane == 0u) g8[0] = s_stage[0];
                    uint4* g16 = reinterpret_cast<uint4*>(g8 + head);
                    for (uint32_t c = lane; c < body; c += 64u) {
                        const unsigned long long x = s_stage[head + 2 * c], y = s_stage[head + 2 * c + 1];
                        g16[c] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
                    }
                    if (lane == 0u && head + 2 * body < units) g8[units - 1] = s_stage[units - 1];
                }
                if (P.dns && is_d) P.dns[base_d + __popcll(m_dn & lmask)] = make_fb_dns(k);
                base_s += ps;
                base_d += (uint32_t)__popcll(m_dn);
            }
        }
        __syncthreads();  // s_cnt / s_excl reuse by the next unit
    }
    const bool owner_last = T > 0u && (T - 1u) % G == blockIdx.x;
    if (!owner_last && tid == 0u && !(FLAGS & kNoLookback)) {
        ast(P.wstat + 2 * blockIdx.x, ((unsigned long long)ep << 56) | a_f | ((unsigned long long)a_t << 28));
        ast(P.wstat + 2 * blockIdx.x + 1, ((unsigned long long)ep << 56) | a_4 | ((unsigned long long)a_b << 28));
    }
}


}  // namespace fbk
