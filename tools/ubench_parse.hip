// ubench_parse.hip -- ablation microbenchmark for the parse kernel (tooling, not product).
// Builds its own binary that includes fb_parse.hip and instantiates ablation variants, plus
// plain streaming read / copy kernels as achievable-bandwidth references.  Variants are timed
// interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
//   build: tools/build_ubench.sh ; run: tools/ubench_parse [config_id] [n] [rotate] [iters]
#include "../flodbadd_amd/csrc/fb_parse.hip"
#ifndef FB_FRAME_WAVES
#define FB_FRAME_WAVES 7
#endif
namespace fbk { constexpr int kExpFrameWaves = FB_FRAME_WAVES; }
#include "parse_experiments.hip"
#ifndef UB_R
#define UB_R fbk::kUnitTiles
#endif
#define UB_TILE (fbk::kTile)

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

extern "C" {
typedef struct fb_synth_cfg {
    uint64_t seed;
    uint32_t n_flows, mode, v6_permille, udp_permille, dns_permille, zipf;
    double zipf_s;
} fb_synth_cfg;
uint64_t fb_synth_plan(const fb_synth_cfg* c, uint64_t first, uint32_t n, uint32_t* offsets);
int fb_synth_fill(const fb_synth_cfg* c, uint64_t first, uint32_t n, const uint32_t* offsets, uint8_t* frames,
                  int n_threads);
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ in, size_t n16, unsigned* sink) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) {
        uint4 v = in[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n_in16,
                                              size_t n_out16) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n_in16; i += (size_t)gridDim.x * 256ull) {
        uint4 v = in[i];
        if (i < n_out16) out[i] = v;
    }
}

__global__ __launch_bounds__(256) void k_hdr_loads(const uint8_t* fr, const uint32_t* off, uint32_t n, uint32_t bytes,
                                                   unsigned* sink) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)fr, (short)0, (int)bytes, 0x00020000);
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t o = off[min(i, n)], o1 = off[min(i + 1u, n)];
    const fbk::u32x4 A = fbk::ld16(rs, o + 10u), B = fbk::ld16(rs, o + 26u), C = fbk::ld16(rs, o + 42u);
    const uint32_t D = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 66u, 0, 0);
    const fbk::u32x4 v = A ^ B ^ C;
    if ((v.x ^ v.y ^ v.z ^ v.w ^ D ^ o1) == 0x9E3779B9u) sink[0] = 1;
}

int main(int argc, char** argv) {
    int cfg_id = argc > 1 ? atoi(argv[1]) : 2;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20);
    int R = argc > 3 ? atoi(argv[3]) : 8;
    int iters = argc > 4 ? atoi(argv[4]) : 200;
    fb_synth_cfg sc;
    memset(&sc, 0, sizeof(sc));
    sc.seed = 0xF10DBADDull ^ (uint64_t)cfg_id;
    sc.n_flows = cfg_id >= 4 ? (1u << 20) : (1u << 16);
    sc.mode = cfg_id == 2 ? 0 : 1;
    sc.v6_permille = cfg_id == 2 ? 0 : 200;
    sc.udp_permille = cfg_id == 2 ? 0 : 300;
    sc.dns_permille = 5;
    sc.zipf_s = 1.1;
    std::vector<uint32_t> offs(n + 1);
    uint64_t bytes = fb_synth_plan(&sc, 0, n, offs.data());
    std::vector<uint8_t> frames(bytes);
    fb_synth_fill(&sc, 0, n, offs.data(), frames.data(), 16);

    // device config: default service bitmap from data/service_ports.bin, filter GlobalOnly
    fbk::DevConfig hc;
    memset(&hc, 0, sizeof(hc));
    FILE* f = fopen("flodbadd_amd/data/service_ports.bin", "rb");
    if (!f || fread(hc.service_bitmap, 1, 8192, f) != 8192) { fprintf(stderr, "bitmap\n"); return 1; }
    fclose(f);
    hc.filter = FB_FILTER_GLOBAL_ONLY;
    fbk::DevConfig* dcfg;
    CK(hipMalloc(&dcfg, sizeof(hc)));
    CK(hipMemcpy(dcfg, &hc, sizeof(hc), hipMemcpyHostToDevice));

    const uint32_t tiles = (n + UB_TILE - 1) / UB_TILE;
    const uint32_t ctiles = (n + fbk::kCtlTile - 1) / fbk::kCtlTile;
    const uint32_t t4 = (n + (fbk::kThreads / 64) * 256 - 1) / ((fbk::kThreads / 64) * 256);
    const uint32_t t2 = (n + (fbk::kThreads / 64) * 128 - 1) / ((fbk::kThreads / 64) * 128);
    // look-back scratch sized for the larger unit count of the kernels (a smaller one let
    // the status words of one kernel overlap its stats slots -> garbage prefixes -> OOB stores)
    const uint32_t stiles = std::max(std::max(tiles, ctiles), std::max(t4, t2));
    const size_t swords = fbk::scratch_words(stiles);
    unsigned long long* status;
    CK(hipMalloc(&status, swords * 8));
    CK(hipMemset(status, 0, swords * 8));
    uint32_t* err;
    CK(hipMalloc(&err, 16));
    CK(hipMemset(err, 0, 16));
    unsigned long long* dbg;
    CK(hipMalloc(&dbg, (size_t)tiles * 32));
    CK(hipMemset(dbg, 0, (size_t)tiles * 32));
    unsigned* sink;
    CK(hipMalloc(&sink, 16));
    struct Buf { uint8_t* fr; uint32_t* off; fb_pkt_out* out; fb_dns_out* dns; fb_batch_stats* st; };
    std::vector<Buf> bufs(R);
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&bufs[r].fr, bytes));
        CK(hipMalloc(&bufs[r].off, (n + 1) * 4ull));
        CK(hipMalloc(&bufs[r].out, n * 56ull));
        CK(hipMalloc(&bufs[r].dns, n * 16ull));
        CK(hipMalloc(&bufs[r].st, sizeof(fb_batch_stats)));
        CK(hipMemcpy(bufs[r].fr, frames.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(bufs[r].off, offs.data(), (n + 1) * 4ull, hipMemcpyHostToDevice));
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint32_t epoch = 0;
    auto params = [&](int r, bool lb, uint32_t nt = 0) {
        if ((nt ? nt : tiles) > stiles) { fprintf(stderr, "scratch too small\n"); exit(2); }
        fbk::ParseParams p;
        p.frames = bufs[r].fr; p.offsets = bufs[r].off; p.out = bufs[r].out; p.dns = bufs[r].dns;
        p.cls = nullptr; p.stats = bufs[r].st; p.cfg = dcfg;
        p.tagg = status; p.wstat = status + stiles;
        p.frames_bytes = (uint32_t)bytes; p.n = n; p.num_tiles = nt ? nt : tiles; p.parsed = nullptr;
        if (lb && ++epoch > 255) { CK(hipStreamSynchronize(s)); CK(hipMemset(status, 0, swords * 8)); CK(hipMemset(err, 0, 16)); epoch = 1; }
        p.epoch = epoch;
        p.error = err + (epoch & 1u); p.error_next = err + ((epoch & 1u) ^ 1u); p.dbg = dbg;
        return p;
    };
    uint64_t caps = 0;
    for (uint32_t i = 0; i < n; ++i) caps += std::min<uint32_t>(offs[i + 1] - offs[i], 128u);
    const double algo = (double)caps + 4.0 * (n + 1) + 56.0 * n;  // upper bound: all emitted
    const char* names[] = {"block", "block_no_lookback", "block_no_store", "block_no_lookback_no_store", "read_frames",
                           "copy_frames_to_out", "header_loads_only", "ctl", "ctl_no_lookback", "ctl_no_store",
                           "ctl_no_lookback_no_store", "block_nonpersistent", "ctl1", "ctl1_no_lookback", "ctl1_no_store",
                           "ctl1_no_lookback_no_store", "2p_u4", "2p_u4_no_lookback", "2p_u4_no_store",
                           "2p_u4_no_lookback_no_store", "2p_u2", "2p_u2_no_lookback"};
    const int NV = 22;
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (fbk::k_parse_block<UB_R, 0>), fbk::kThreads, 0));
    int cbpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&cbpc, (fbk::k_parse_ctl<fbk::kCtlU, 0>), fbk::kCtlThreads, 0));
    cbpc = std::min(cbpc, std::max(1, 24 / (fbk::kCtlThreads / 64)));
    int c1bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&c1bpc, (fbk::k_parse_ctl1<fbk::kCtlU, 0, false, 2>), fbk::kCtlThreads, 0));
    c1bpc = std::min(c1bpc, std::max(1, 24 / (fbk::kCtlThreads / 64)));
    printf("{\"ctl_blocks_per_cu\": %d, \"ctl1_blocks_per_cu\": %d, \"ctl_units\": %u}\n", cbpc, c1bpc, ctiles);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    printf("{\"blocks_per_cu_api\": %d, \"cus\": %d, \"tiles\": %u}\n", bpc, prop.multiProcessorCount, tiles);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 3;
    const int blimit = std::min(bpc, std::max(1, 24 / (fbk::kThreads / 64)));
    int pbpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pbpc, (fbk::k_parse_2p<4, 0>), fbk::kThreads, 0));
    pbpc = std::min(pbpc, std::max(1, 24 / (fbk::kThreads / 64)));
    const int maxb = std::max(std::max(std::max(blimit, cbpc), c1bpc), pbpc);
    for (int bpcu = 1; bpcu <= maxb; ++bpcu) {
        const uint32_t grid = std::min<uint32_t>(tiles, (uint32_t)(bpcu * prop.multiProcessorCount));
        const uint32_t cgrid = std::min<uint32_t>(ctiles, (uint32_t)(std::min(bpcu, cbpc) * prop.multiProcessorCount));
        const uint32_t p4grid = std::min<uint32_t>(t4, (uint32_t)(std::min(bpcu, pbpc) * prop.multiProcessorCount));
        const uint32_t p2grid = std::min<uint32_t>(t2, (uint32_t)(std::min(bpcu, pbpc) * prop.multiProcessorCount));
        const uint32_t c1grid = std::min<uint32_t>(ctiles, (uint32_t)(std::min(bpcu, c1bpc) * prop.multiProcessorCount));
        std::vector<double> best(NV, 1e30), sum(NV, 0.0);
        for (int round = 0; round < rounds; ++round) {
            for (int v = 0; v < NV; ++v) {
                if (((v >= 4 && v <= 6) || v == 11) && bpcu > 1) continue;
                if (v >= 7 && v <= 10 && bpcu > cbpc) continue;
            if (v >= 12 && v <= 15 && bpcu > c1bpc) continue;
            if (v >= 16 && bpcu > pbpc) continue;
                if (v >= 12 && v <= 15 && bpcu > c1bpc) continue;
                if (v >= 16 && bpcu > pbpc) continue;
            if (v <= 3 && bpcu > blimit) continue;
                if (v <= 3 && bpcu > blimit) continue;
                for (int warm = -10; warm < iters; ++warm) {
                    if (warm == 0) CK(hipEventRecord(e0, s));
                    int r = (warm + 100) % R;
                    switch (v) {
                    case 0: hipLaunchKernelGGL((fbk::k_parse_block<UB_R, 0>), dim3(grid), dim3(fbk::kThreads), 0, s, params(r, true)); break;
                    case 1: hipLaunchKernelGGL((fbk::k_parse_block<UB_R, fbk::kNoLookback>), dim3(grid), dim3(fbk::kThreads), 0, s, params(r, true)); break;
                    case 2: hipLaunchKernelGGL((fbk::k_parse_block<UB_R, fbk::kNoStore>), dim3(grid), dim3(fbk::kThreads), 0, s, params(r, true)); break;
                    case 3: hipLaunchKernelGGL((fbk::k_parse_block<UB_R, fbk::kNoLookback | fbk::kNoStore>), dim3(grid), dim3(fbk::kThreads), 0, s, params(r, true)); break;
                    case 4: hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, bytes / 16, sink); break;
                    case 5: hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, (uint4*)bufs[r].out, bytes / 16, n * 56ull / 16); break;
                    case 7: hipLaunchKernelGGL((fbk::k_parse_ctl<fbk::kCtlU, 0>), dim3(cgrid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 8: hipLaunchKernelGGL((fbk::k_parse_ctl<fbk::kCtlU, fbk::kNoLookback>), dim3(cgrid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 9: hipLaunchKernelGGL((fbk::k_parse_ctl<fbk::kCtlU, fbk::kNoStore>), dim3(cgrid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 10: hipLaunchKernelGGL((fbk::k_parse_ctl<fbk::kCtlU, fbk::kNoLookback | fbk::kNoStore>), dim3(cgrid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 12: hipLaunchKernelGGL((fbk::k_parse_ctl1<fbk::kCtlU, 0, false, 2>), dim3(c1grid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 13: hipLaunchKernelGGL((fbk::k_parse_ctl1<fbk::kCtlU, fbk::kNoLookback, false, 2>), dim3(c1grid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 14: hipLaunchKernelGGL((fbk::k_parse_ctl1<fbk::kCtlU, fbk::kNoStore, false, 2>), dim3(c1grid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 15: hipLaunchKernelGGL((fbk::k_parse_ctl1<fbk::kCtlU, fbk::kNoLookback | fbk::kNoStore, false, 2>), dim3(c1grid), dim3(fbk::kCtlThreads), 0, s, params(r, true, ctiles)); break;
                    case 16: hipLaunchKernelGGL((fbk::k_parse_2p<4, 0>), dim3(p4grid), dim3(fbk::kThreads), 0, s, params(r, true, t4)); break;
                    case 17: hipLaunchKernelGGL((fbk::k_parse_2p<4, fbk::kNoLookback>), dim3(p4grid), dim3(fbk::kThreads), 0, s, params(r, true, t4)); break;
                    case 18: hipLaunchKernelGGL((fbk::k_parse_2p<4, fbk::kNoStore>), dim3(p4grid), dim3(fbk::kThreads), 0, s, params(r, true, t4)); break;
                    case 19: hipLaunchKernelGGL((fbk::k_parse_2p<4, fbk::kNoLookback | fbk::kNoStore>), dim3(p4grid), dim3(fbk::kThreads), 0, s, params(r, true, t4)); break;
                    case 20: hipLaunchKernelGGL((fbk::k_parse_2p<2, 0>), dim3(p2grid), dim3(fbk::kThreads), 0, s, params(r, true, t2)); break;
                    case 21: hipLaunchKernelGGL((fbk::k_parse_2p<2, fbk::kNoLookback>), dim3(p2grid), dim3(fbk::kThreads), 0, s, params(r, true, t2)); break;
                    case 11: hipLaunchKernelGGL((fbk::k_parse_block<UB_R, 0>), dim3(tiles), dim3(fbk::kThreads), 0, s, params(r, true)); break;
                    case 6: hipLaunchKernelGGL(k_hdr_loads, dim3((n + 255) / 256), dim3(256), 0, s, bufs[r].fr, bufs[r].off, n, (uint32_t)bytes, sink); break;
                    }
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                double us = ms * 1e3 / iters;
                best[v] = std::min(best[v], us);
                sum[v] += us;
            }
        }
        for (int v = 0; v < NV; ++v) {
            if (((v >= 4 && v <= 6) || v == 11) && bpcu > 1) continue;
            if (v >= 7 && v <= 10 && bpcu > cbpc) continue;
            if (v >= 12 && v <= 15 && bpcu > c1bpc) continue;
            if (v >= 16 && bpcu > pbpc) continue;
            if (v <= 3 && bpcu > blimit) continue;
            double us = sum[v] / rounds;
            double gbs = v == 4 ? bytes / (best[v] * 1e3) : (v == 5 ? (bytes + n * 56.0) / (best[v] * 1e3) : algo / (best[v] * 1e3));
            printf("{\"variant\": \"%s\", \"blocks_per_cu\": %d, \"grid\": %u, \"us_mean\": %.2f, \"us_best\": %.2f, \"Gpps\": %.2f, \"GBs\": %.1f}\n",
                   names[v], bpcu, grid, us, best[v], n / (best[v] * 1e3), gbs);
        }
        fflush(stdout);
    }
    {
        // stamped run (diagnostic build of the same kernel)
        const uint32_t grid = std::min<uint32_t>(tiles, (uint32_t)(blimit * prop.multiProcessorCount));
        for (int w = 0; w < 5; ++w)
            hipLaunchKernelGGL((fbk::k_parse_block<UB_R, fbk::kStamps>), dim3(grid), dim3(fbk::kThreads), 0, s, params(w % R, true));
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> st(tiles * 4ull);
        CK(hipMemcpy(st.data(), dbg, st.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (uint32_t t = 0; t < tiles; ++t) t0 = std::min(t0, st[t * 4]);
        const uint32_t W = grid;
        const uint32_t nround = (tiles + W - 1) / W;
        for (uint32_t r = 0; r < nround; ++r) {
            std::vector<double> cl, li, ld, wait, sp;
            for (uint32_t t = r * W; t < std::min(tiles, (r + 1) * W); ++t) {
                cl.push_back((st[t * 4] - t0) * 0.01);
                li.push_back((st[t * 4 + 1] - t0) * 0.01);
                ld.push_back((st[t * 4 + 2] - t0) * 0.01);
                wait.push_back((st[t * 4 + 2] - st[t * 4]) * 0.01);
                sp.push_back((double)st[t * 4 + 3]);
            }
            auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
            printf("{\"round\": %u, \"classified_us\": [%.2f, %.2f, %.2f], \"lb_issue_us\": [%.2f, %.2f, %.2f], \"lb_done_us\": [%.2f, %.2f, %.2f], \"lb_wait_us\": [%.2f, %.2f, %.2f], \"spins\": [%.0f, %.0f, %.0f]}\n",
                   r, q(cl, 0.0), q(cl, 0.5), q(cl, 1.0), q(li, 0.0), q(li, 0.5), q(li, 1.0), q(ld, 0.0), q(ld, 0.5), q(ld, 1.0),
                   q(wait, 0.0), q(wait, 0.5), q(wait, 1.0), q(sp, 0.0), q(sp, 0.5), q(sp, 1.0));
        }
    }
    {
        const uint32_t grid = std::min<uint32_t>(tiles, (uint32_t)(blimit * prop.multiProcessorCount));
        hipLaunchKernelGGL((fbk::k_parse_block<UB_R, 0>), dim3(grid), dim3(fbk::kThreads), 0, s, params(0, true));
        CK(hipStreamSynchronize(s));
    }
    unsigned errw[2] = {0, 0};
    CK(hipMemcpy(errw, err, 8, hipMemcpyDeviceToHost));
    fb_batch_stats st;
    CK(hipMemcpy(&st, bufs[0].st, sizeof(st), hipMemcpyDeviceToHost));
    printf("{\"config\": %d, \"n\": %u, \"bytes\": %llu, \"rotate\": %d, \"err\": [%u, %u], \"n_session\": %llu, \"n_dns\": %llu, \"stats_error\": %llu}\n",
           cfg_id, n, (unsigned long long)bytes, R, errw[0], errw[1], (unsigned long long)st.n_session, (unsigned long long)st.n_dns,
           (unsigned long long)st.error);
    return 0;
}
