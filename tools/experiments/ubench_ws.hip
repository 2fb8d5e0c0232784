// ubench_ws.hip -- timing of the segmented parse kernel (tooling, not product).  Includes the
// product kernel source and times, interleaved in one process:
//   read / copy   plain streaming read of the frame buffer / read frames + write 56 B per frame
//   seg           the product kernel (k_parse_seg<false>)
// (The round-2 ablations -- no stores, no classification, per-wave stamps -- were template flags
// of the product kernel; they are no longer in the product source.  DESIGN.md keeps their numbers.)
//   build: tools/experiments/build_ubench_ws.sh ; run: tools/ubench_ws [config_id] [n] [rotate] [iters]
#include "../flodbadd_amd/csrc/fb_parse.hip"

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

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
            exit(1);                                                                           \
        }                                                                                      \
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
    const int cfg_id = argc > 1 ? atoi(argv[1]) : 2;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20);
    const int R = argc > 3 ? atoi(argv[3]) : 8;
    const int iters = argc > 4 ? atoi(argv[4]) : 200;
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
    const uint64_t bytes = fb_synth_plan(&sc, 0, n, offs.data());
    std::vector<uint8_t> frames(bytes);
    fb_synth_fill(&sc, 0, n, offs.data(), frames.data(), 16);

    fbk::DevConfig hc;
    memset(&hc, 0, sizeof(hc));
    FILE* f = fopen("flodbadd_amd/data/service_ports.bin", "rb");
    if (!f || fread(hc.service_bitmap, 1, 8192, f) != 8192) { fprintf(stderr, "bitmap\n"); return 1; }
    fclose(f);
    hc.filter = FB_FILTER_GLOBAL_ONLY;
    fbk::DevConfig* dcfg;
    CK(hipMalloc(&dcfg, sizeof(hc)));
    CK(hipMemcpy(dcfg, &hc, sizeof(hc), hipMemcpyHostToDevice));

    unsigned long long* tick;
    CK(hipMalloc(&tick, fbk::kTickWords * 8));
    CK(hipMemset(tick, 0, fbk::kTickWords * 8));
    uint32_t* err;
    CK(hipMalloc(&err, 16));
    CK(hipMemset(err, 0, 16));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    unsigned* sink;
    CK(hipMalloc(&sink, 16));
    struct Buf { uint8_t* fr; uint32_t* off; fb_pkt_out* out; fb_dns_out* dns; fb_batch_stats* st; };
    std::vector<Buf> bufs(R);
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&bufs[r].fr, bytes));
        CK(hipMalloc(&bufs[r].off, (n + 1) * 4ull));
        CK(hipMalloc(&bufs[r].out, ((n + 63) / 64) * 3584ull));
        CK(hipMalloc(&bufs[r].dns, n * 16ull));
        CK(hipMalloc(&bufs[r].st, sizeof(fb_batch_stats)));
        CK(hipMemcpy(bufs[r].fr, frames.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(bufs[r].off, offs.data(), (n + 1) * 4ull, hipMemcpyHostToDevice));
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint32_t launch = 0;
    auto params = [&]() {
        fbk::ParseParams p;
        memset(&p, 0, sizeof(p));
        p.cfg = dcfg;
        p.tick = tick;
        ++launch;
        p.error = err + (launch & 1u); p.error_next = err + ((launch & 1u) ^ 1u);
        return p;
    };
    auto sb1 = [&](int r, uint32_t* seg) {  // one-batch launch descriptor of k_parse_seg
        fbk::SegBatches sb;
        memset(&sb, 0, sizeof(sb));
        sb.count = 1;
        sb.b[0].frames = bufs[r].fr; sb.b[0].offsets = bufs[r].off; sb.b[0].out = bufs[r].out; sb.b[0].seg = seg;
        sb.b[0].cls = nullptr; sb.b[0].stats = bufs[r].st; sb.b[0].n = n; sb.b[0].frames_bytes = (uint32_t)bytes;
        sb.total_segs = (n + 63u) / 64u;
        return sb;
    };
    uint64_t caps = 0;
    for (uint32_t i = 0; i < n; ++i) caps += std::min<uint32_t>(offs[i + 1] - offs[i], 128u);
    const double algo = (double)caps + 4.0 * (n + 1) + 56.0 * n;
    printf("{\"cus\": %d}\n", prop.multiProcessorCount);
    const char* names[] = {"read", "copy", "seg"};
    const int NV = 3;
    int sbpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&sbpc, (fbk::k_parse_seg<false>), fbk::kSegThreads, 0));
    const uint32_t nseg = (n + 63) / 64;
    const uint32_t sgrid = std::min<uint32_t>((uint32_t)(sbpc * prop.multiProcessorCount),
                                              (nseg + fbk::kSegWaves - 1) / fbk::kSegWaves);
    uint32_t* dseg;
    CK(hipMalloc(&dseg, nseg * 4ull));
    printf("{\"seg_blocks_per_cu\": %d, \"seg_grid\": %u}\n", sbpc, sgrid);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> best(NV, 1e30), sum(NV, 0.0);
    const int rounds = 3;
    for (int round = 0; round < rounds; ++round) {
        for (int v = 0; v < NV; ++v) {
            for (int it = -10; it < iters; ++it) {
                if (it == 0) CK(hipEventRecord(e0, s));
                const int r = (it + 100) % R;
                switch (v) {
                case 0: hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, bytes / 16, sink); break;
                case 1: hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, s, (const uint4*)bufs[r].fr, (uint4*)bufs[r].out, bytes / 16, n * 56ull / 16); break;
                case 2: hipLaunchKernelGGL((fbk::k_parse_seg<false, 0>), dim3(sgrid), dim3(fbk::kSegThreads), 0, s, params(), sb1(r, dseg)); break;
                }
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            best[v] = std::min(best[v], us);
            sum[v] += us;
        }
    }
    for (int v = 0; v < NV; ++v) {
        const double gbs = v == 0 ? bytes / (best[v] * 1e3) : (v == 1 ? (bytes + n * 56.0) / (best[v] * 1e3) : algo / (best[v] * 1e3));
        printf("{\"variant\": \"%s\", \"us_mean\": %.2f, \"us_best\": %.2f, \"Gpps\": %.2f, \"GBs\": %.1f}\n", names[v],
               sum[v] / rounds, best[v], n / (best[v] * 1e3), gbs);
    }
    hipLaunchKernelGGL((fbk::k_parse_seg<false, 0>), dim3(sgrid), dim3(fbk::kSegThreads), 0, s, params(), sb1(0, dseg));
    CK(hipStreamSynchronize(s));
    unsigned errw[2] = {0, 0};
    CK(hipMemcpy(errw, err, 8, hipMemcpyDeviceToHost));
    fb_batch_stats bs;
    CK(hipMemcpy(&bs, bufs[0].st, sizeof(bs), hipMemcpyDeviceToHost));
    printf("{\"config\": %d, \"n\": %u, \"bytes\": %llu, \"rotate\": %d, \"err\": [%u, %u], \"n_session\": %llu, \"n_dns\": %llu, \"stats_error\": %llu}\n",
           cfg_id, n, (unsigned long long)bytes, R, errw[0], errw[1], (unsigned long long)bs.n_session,
           (unsigned long long)bs.n_dns, (unsigned long long)bs.error);
    return 0;
}
