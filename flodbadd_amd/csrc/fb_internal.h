// fb_internal.h -- definitions shared by the gfx950 kernels and the C-ABI host code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flodbadd_gpu.h"

namespace fbk {

// Packets per tile = kThreads * kRounds; one wavefront lane per packet per round.
constexpr int kThreads = 256;
constexpr int kRounds = 2;
constexpr int kPRounds = kRounds;  // persistent kernel (same tile size)
constexpr int kTile = kThreads * kRounds;
// Tiles per look-back group (two-level decoupled look-back, fb_parse.hip lookback()).
constexpr int kGroup = 32;

// Look-back scratch (one allocation per context, zeroed when the 8-bit epoch wraps):
//   tagg[tiles]          tile aggregate          [epoch:8 | n_dns:28 | n_session:28]
//   ginc[groups]         group inclusive prefix  [epoch:8 | n_dns:28 | n_session:28]
//   gpre[groups]         group exclusive prefix  [epoch:8 | n_dns:28 | n_session:28]
//   gacc[2][groups]      group accumulator       [arrivals:8 | n_dns:28 | n_session:28]
//   gstat[2][groups][2]  group stats             [arrivals:8 | n_tcp:28 | n_filtered:28],
//                                                [arrivals:8 | n_bad:28 | n_ipv4:28]
// Epoch-tagged words need no per-launch zeroing; the two accumulator parities alternate
// between launches and each launch zeroes the parity the next one uses.
constexpr uint32_t kMaxEpoch = 255;
inline uint64_t scratch_words(uint64_t tiles) {
    const uint64_t groups = (tiles + kGroup - 1) / kGroup;
    return tiles + groups + groups + 2 * groups + 4 * groups;
}

// Device-resident configuration (uploaded lazily, stream-ordered, before a launch).
struct LanV6 {
    uint32_t net[4];
    uint32_t mask[4];
};
struct DevConfig {
    uint32_t service_bitmap[FB_SERVICE_BITMAP_BYTES / 4];  // bit p <=> name(p) != ""
    uint32_t filter;
    uint32_t n_lan_v6;
    uint32_t n_own;
    uint32_t pad;
    LanV6 lan_v6[FB_MAX_LAN_V6];
    fb_ip own[FB_MAX_OWN_IPS];
};

struct ParseParams {
    const uint8_t* frames;
    const uint32_t* offsets;
    fb_pkt_out* out;
    fb_dns_out* dns;
    uint8_t* cls;
    fb_batch_stats* stats;
    unsigned long long* tagg;
    unsigned long long* ginc;
    unsigned long long* gpre;
    unsigned long long* gacc;   // [2][max_groups]
    unsigned long long* gstat;  // [2][max_groups][2]
    uint32_t max_groups;
    const DevConfig* cfg;
    uint32_t frames_bytes;  // min(frames_bytes, 2^32 - 1)
    uint32_t n;
    uint32_t num_tiles;
    uint32_t epoch;
    uint32_t* error;  // set nonzero when a bounded spin expires
    unsigned long long* dbg;  // diagnostic timestamps (ablation builds only; nullptr in product)
};

// Flow table: 128-byte slots (one L2 line).  tag: 0 empty, 1 being inserted, else
// (hash | 2).  Key words 8..47, counters 48..95 (fb_flow_rec order).
struct FlowSlot {
    unsigned long long tag;
    uint32_t key[10];
    unsigned long long cnt[6];  // outbound_bytes, inbound_bytes, orig_pkts, resp_pkts,
                                // orig_ip_bytes, resp_ip_bytes
    unsigned long long pad[4];
};
static_assert(sizeof(FlowSlot) == 128, "flow slot must be one 128-B line");

struct FlowParams {
    const fb_pkt_out* recs;
    fb_batch_stats* stats;  // n_session read from here; new/updated accumulated
    FlowSlot* table;
    unsigned long long mask;  // capacity - 1
    unsigned long long* partials;  // 2 per block: new, updated
    uint32_t* error;
    uint32_t max_recs;
};

// Launchers (fb_parse.hip / fb_flow.hip).
hipError_t launch_parse_classify(const ParseParams& p, hipStream_t s);
hipError_t launch_parse_persistent(const ParseParams& p, uint32_t grid, hipStream_t s);
hipError_t occupancy_parse_persistent(int* blocks_per_cu);
hipError_t launch_flow_update(const FlowParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_flow_finish(fb_batch_stats* stats, const unsigned long long* partials,
                              uint32_t nblk, uint32_t* error, hipStream_t s);
hipError_t launch_flow_export(const FlowSlot* table, unsigned long long cap, fb_flow_rec* out,
                              unsigned long long out_cap, unsigned long long* d_n,
                              hipStream_t s);
hipError_t launch_flow_count(const FlowSlot* table, unsigned long long cap,
                             unsigned long long* d_n, hipStream_t s);

}  // namespace fbk
