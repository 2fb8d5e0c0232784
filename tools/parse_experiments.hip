// parse_experiments.hip -- kernel variants that were measured and NOT adopted (tooling only;
// included by tools/ubench_parse.hip after flodbadd_amd/csrc/fb_parse.hip).
//
// k_parse_pipe: frame waves + a control wave, look-back of round k overlapped with the stores of
// round k-1 and the loads of round k+1.  Measured (C2, 1M x 64 B, 8 rotating batches, MI355X):
// 71 us at 7 frame waves x 2 blocks/CU vs 44 us for k_parse_block -- the loop-carried
// prefetch makes every round wait for its own store completions and load latency.
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


}  // namespace fbk
