// ubench_parse.hip -- ablation microbenchmark for the parse kernel (tooling, not product).
// Builds its own binary that includes fb_parse.hip and instantiates ablation variants, plus
// plain streaming read / copy kernels as achievable-bandwidth references.  Variants are timed
// interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
//   build: tools/build_ubench.sh ; run: tools/ubench_parse [config_id] [n] [rotate] [iters]
#include "../flodbadd_amd/csrc/fb_parse.hip"
#ifndef UB_R
#define UB_R fbk::kRounds
#endif
#define UB_TILE (fbk::kThreads * UB_R)

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
    const uint32_t stiles = (tiles + fbk::kGroup - 1) / fbk::kGroup * fbk::kGroup;
    const size_t swords = fbk::scratch_words(stiles);
    unsigned long long* status;
    CK(hipMalloc(&status, swords * 8));
    CK(hipMemset(status, 0, swords * 8));
    uint32_t* err;
    CK(hipMalloc(&err, 16));
    CK(hipMemset(err, 0, 16));
    unsigned long long* dbg;
    CK(hipMalloc(&dbg, (size_t)tiles * 64));
    CK(hipMemset(dbg, 0, (size_t)tiles * 64));
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
    auto params = [&](int r, bool lb) {
        fbk::ParseParams p;
        p.frames = bufs[r].fr; p.offsets = bufs[r].off; p.out = bufs[r].out; p.dns = bufs[r].dns;
        p.cls = nullptr; p.stats = bufs[r].st; p.cfg = dcfg;
        p.tagg = status; p.ginc = status + stiles; p.gpre = p.ginc + stiles / fbk::kGroup; p.gacc = p.gpre + stiles / fbk::kGroup;
        p.gstat = p.gacc + 2 * (stiles / fbk::kGroup); p.max_groups = stiles / fbk::kGroup;
        p.frames_bytes = (uint32_t)bytes; p.n = n; p.num_tiles = tiles; p.error = err; p.dbg = dbg;
        if (lb && ++epoch > 255) { CK(hipStreamSynchronize(s)); CK(hipMemset(status, 0, swords * 8)); epoch = 1; }
        p.epoch = epoch;
        return p;
    };
    uint64_t caps = 0;
    for (uint32_t i = 0; i < n; ++i) caps += std::min<uint32_t>(offs[i + 1] - offs[i], 128u);
    const double algo = (double)caps + 4.0 * (n + 1) + 56.0 * n;  // upper bound: all emitted
    const char* names[] = {"product", "no_lookback", "no_store", "loads_classify_only", "read_frames", "copy_frames_to_out",
                           "header_loads_only", "coalesced_loads_only", "persistent"};
    const int NV = 9;
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (fbk::k_parse_persistent<UB_R, 0>), fbk::kPThreads, 0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const uint32_t pgrid = std::min<uint32_t>(tiles, (uint32_t)(std::max(bpc - 1, 1) * prop.multiProcessorCount));
    printf("{\"persistent_blocks_per_cu_api\": %d, \"grid\": %u, \"cus\": %d}\n", bpc, pgrid, prop.multiProcessorCount);
    std::vector<double> best(NV, 1e30), sum(NV, 0.0);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 5;
    for (int round = 0; round < rounds; ++round) {
        for (int v = 0; v < NV; ++v) {
            for (int warm = -10; warm < iters; ++warm) {
                if (warm == 0) CK(hipEventRecord(e0, s));
                int r = (warm + 100) % R;
                switch (v) {
                case 0: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, 0>), dim3(tiles), dim3(256), 0, s, params(r, true)); break;
                case 1: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kNoLookback>), dim3(tiles), dim3(256), 0, s, params(r, false)); break;
                case 2: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kNoStore>), dim3(tiles), dim3(256), 0, s, params(r, true)); break;
                case 3: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kNoLookback | fbk::kNoStore>), dim3(tiles), dim3(256), 0, s, params(r, true)); break;
                case 4: hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, bytes / 16, sink); break;
                case 6: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kLoadsOnly>), dim3(tiles), dim3(256), 0, s, params(r, false)); break;
                case 7: hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kLoadsOnly | fbk::kCoalesced>), dim3(tiles), dim3(256), 0, s, params(r, false)); break;
                case 8: hipLaunchKernelGGL((fbk::k_parse_persistent<UB_R, 0>), dim3(pgrid), dim3(fbk::kPThreads), 0, s, params(r, true)); break;
                case 5: hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, (uint4*)bufs[r].out, bytes / 16, n * 56ull / 16); break;
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
    // ---- timeline of one stamped launch (after warm-up) ----
    for (int w = 0; w < 5; ++w)
        hipLaunchKernelGGL((fbk::k_parse_classify<UB_R, fbk::kStamps>), dim3(tiles), dim3(256), 0, s, params(w % R, true));
    CK(hipStreamSynchronize(s));
    {
        std::vector<unsigned long long> st(tiles * 8ull);
        CK(hipMemcpy(st.data(), dbg, st.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (uint32_t t = 0; t < tiles; ++t) t0 = std::min(t0, st[t * 8]);
        const char* ph[] = {"entry", "classified", "published", "lookback_done", "end"};
        for (int k = 0; k < 5; ++k) {
            std::vector<double> v;
            for (uint32_t t = 0; t < tiles; ++t) v.push_back((st[t * 8 + k] - t0) * 0.01);  // 100 MHz -> us
            std::vector<double> sv = v;
            std::sort(sv.begin(), sv.end());
            printf("{\"stamp\": \"%s\", \"us_min\": %.2f, \"us_p10\": %.2f, \"us_med\": %.2f, \"us_p90\": %.2f, \"us_max\": %.2f, \"first_tiles\": [%.2f, %.2f, %.2f], \"last_tile\": %.2f}\n",
                   ph[k], sv[0], sv[sv.size() / 10], sv[sv.size() / 2], sv[sv.size() * 9 / 10], sv.back(), v[0], v[1], v[2], v.back());
        }
    }
    unsigned e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    fb_batch_stats st;
    CK(hipMemcpy(&st, bufs[0].st, sizeof(st), hipMemcpyDeviceToHost));
    printf("{\"config\": %d, \"n\": %u, \"bytes\": %llu, \"rotate\": %d, \"err\": %u, \"n_session\": %llu, \"n_dns\": %llu}\n",
           cfg_id, n, (unsigned long long)bytes, R, e, (unsigned long long)st.n_session, (unsigned long long)st.n_dns);
    for (int v = 0; v < NV; ++v) {
        double us = sum[v] / rounds;
        double gbs = v == 4 ? bytes / (best[v] * 1e3) : (v == 5 ? (bytes + n * 56.0) / (best[v] * 1e3) : algo / (best[v] * 1e3));
        printf("{\"variant\": \"%s\", \"us_mean\": %.2f, \"us_best\": %.2f, \"Gpps\": %.2f, \"GBs\": %.1f}\n", names[v], us,
               best[v], n / (best[v] * 1e3), gbs);
    }
    return 0;
}
