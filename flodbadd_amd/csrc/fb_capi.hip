// fb_capi.hip -- C ABI (include/flodbadd_gpu.h) over the gfx950 kernels.
//
// Host-side counterpart of the reference capture task's per-packet calls
// (src/capture.rs:1036-1061 / 1219-1249): a context owns the device-resident configuration
// (service-port bitmap, filter, IPv6 LAN prefixes, own IPs), the look-back scratch, the flow
// table and (lazily) host-mode staging buffers.  Every entry point returns an fb_err code;
// nothing aborts.  No CPU fallback exists: without a gfx950 device fb_create fails.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "fb_host.h"
#include "fb_internal.h"
#include "service_ports_default.inc"  // kDefaultServiceBitmap[8192] (generated at build time)

using namespace fbk;

namespace fbk {

static thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace fbk

// Update scratch of one table update (K1 bucketing -> K1c -> K1t -> K2).  Two sets: the pipelined
// call buckets batch k (on the caller's stream, right after its parse) into set k & 1 while the
// update stream applies batch k - 1 from the other set.
struct UpdScratch {
    uint32_t* entries = nullptr;   // [flow_recs] bucketed record slots (or combined ids)
    FlowEntry* comb = nullptr;     // k_flow_combine entries (2 units each), comb_cap of them
    uint32_t* rows = nullptr;      // [flow_chunks][flow_parts]
    uint32_t* cols = nullptr;      // [flow_parts][flow_chunks]
    uint32_t* rows_h = nullptr;    // [flow_chunks][flow_parts] combined groups' rows before k_flow_combine
    uint32_t* e_orig = nullptr;    // [flow_recs] combined groups' original entry words (history)
    uint2* e_sort = nullptr;       // [flow_recs] combined groups' records in record order (history)
    uint32_t* hot = nullptr;       // [flow_recs / 16 + 16] hot groups for k_flow_combine
    uint32_t* ctl = nullptr;       // [4] its counters (FlowParams::ctl)
    uint32_t* order = nullptr;     // [flow_parts + kK2Lead + 1] K2's partition order (FlowParams::order)
};

struct fb_ctx {
    int device = 0;
    DevConfig* h_cfg = nullptr;  // host shadow
    DevConfig* d_cfg = nullptr;
    bool cfg_dirty = true;
    unsigned long long* d_tick = nullptr;  // [kTickWords] k_parse_seg stats words
    bool need_reset = true;       // zero the tick + error words before the next launch
    uint32_t epoch = 0;           // parse launches so far: its parity picks the launch's error word
    uint32_t seg_grid = 0;        // streaming segmented kernel: co-resident blocks
    uint32_t seg_grid_async = 0;  // ... in the pipelined call: FB_ASYNC_BPC blocks per CU (not the full
                                  // grid), so the previous batch's table update keeps part of each CU
    uint32_t* d_error = nullptr;  // [4] error words, indexed by launch & 3 (a launch clears the next one's;
                                  // a pipelined update still writes the one two launches back)
    // dense output (fb_parse_classify_dev & co., fb_seg_compact_dev): segment counts + their scan
    uint32_t* d_cseg = nullptr;            // [cseg_cap] segment counts (dense pass 1)
    unsigned long long* d_cpre = nullptr;  // [cseg_cap] batch-wide offset of every segment
    unsigned long long* d_cstatus = nullptr;  // [seg_scan_tiles(cseg_cap)] scan look-back words
    uint32_t* d_cticket = nullptr;            // scan ticket counter
    uint32_t scan_epoch = 0;                  // epoch of the last scan (0: status needs zeroing)
    uint64_t cseg_cap = 0;                    // segments
    // single-pass dense output (k_parse_dense): per-tile look-back words, epoch, grid, and the
    // look-back's polls before it computes a late predecessor's sums itself (fb_debug_set
    // FB_DEBUG_DENSE_STEAL_POLLS; tests set 0 to force that path)
    unsigned long long* d_dstatus = nullptr;  // [cseg_cap / parse_dense_tile_segs() + 1]
    uint32_t dense_epoch = 0;                 // epoch of the last launch (0: status needs zeroing)
    uint32_t dense_grid = 0;
    uint32_t steal_polls = 1u << 12;
    unsigned long long dn_skew = 0ull;  // FB_DEBUG_DENSE_OFFSET_SKEW: fault injection (k_parse_dense copy bounds)
    hipEvent_t stage_event = nullptr;  // fb_set_stage_event (caller-owned): recorded between the
                                       // parse and the update of fb_process[_seg]_dev
    // flow table
    FlowSlot* d_table = nullptr;
    uint64_t table_cap = 0;
    uint32_t flow_parts = 0;        // partitions of kFlowSlots slots
    uint32_t flow_shift = 64;       // 64 - log2(flow_parts)
    UpdScratch us[2];               // update scratch sets (set 1: pipelined calls only, allocated lazily)
    uint32_t comb_cap = 0;
    uint64_t flow_recs = 0;         // scratch capacity (multiple of kFlowChunk)
    uint32_t last_n = 0;            // packets of the last parse launch (bounds its records)
    unsigned long long* d_partials = nullptr;  // [3 * flow_parts] per-partition new / updated / occupied
    // growth: the occupancy each update reports in host-mapped memory, updates issued
    FlowMailbox* h_mbox = nullptr;  // pinned, host-mapped (written by k_flow_finish)
    FlowMailbox* d_mbox = nullptr;  // its device address
    uint64_t upd_seq = 0;           // table updates issued (the mailbox's seq counts them from 1)
    uint64_t grown_seq = 0;         // upd_seq at the last growth (older reports describe the old geometry)
    uint64_t clear_seq = 0;         // upd_seq at the last fb_flow_clear (older reports are void)
    uint64_t generation = 0;        // growths so far
    bool grow = true;               // FB_CFG_FIXED_TABLE clears it
    uint32_t* d_remap = nullptr;    // the last growth's old -> new slot map
    uint4* d_char_call = nullptr;   // [table_cap] first update call of S s H h per slot (the merge's)
    // timed contexts (FB_CFG_TIMED, fb_time.hip): the time plane, the next update's frame times, the
    // capture-time pass's scratch (its last use: ev_tscratch)
    bool timed = false;
    FlowTime* d_time = nullptr;               // [table_cap]
    const unsigned long long* next_ts = nullptr;
    void* d_tscratch = nullptr;
    uint64_t tscratch_bytes = 0;
    hipEvent_t ev_tscratch = nullptr;
    void* d_mscratch = nullptr;     // multi-GPU merge scratch (export owner counts / merge tables)
    hipEvent_t ev_mscratch = nullptr;  // after the last export / merge that used d_mscratch (either may
                                       // run on any stream: the next use waits for it)
    uint64_t mscratch_bytes = 0;
    uint64_t remap_n = 0;
    unsigned long long* d_n = nullptr;
    // ordered per-flow state: update calls since create/clear, table slot of each record slot
    uint32_t flow_batch = 0;
    uint32_t* d_hword = nullptr;          // [flow_recs] K2's history word per entry
    uint32_t* d_rec_part = nullptr;       // [flow_recs] partition per record slot (fb_process_seg_dev)
    const fb_pkt_out* part_recs = nullptr;  // the records part_buf was written for (one update)
    uint32_t* part_buf = nullptr;           // the partition buffer the last fused parse wrote
    uint32_t* part_target = nullptr;        // the buffer the next fused parse writes (null: d_rec_part)
    uint4* d_rec_ent = nullptr;             // [flow_recs] update entry (UpdEnt, 64 B) per record slot
    uint4* d_rec_ent2 = nullptr;            // ... of the odd async batches
    uint4* ent_buf = nullptr;               // the entries the last fused parse wrote (with part_buf)
    uint4* ent_target = nullptr;            // the entries the next fused parse writes (null: d_rec_ent)
    bool emit_records = true;               // fb_set_session_records: fused calls store SESSION records
    // fb_process_seg_async_dev: updates on the context's own stream, one batch behind the parses
    hipStream_t upd = nullptr;
    hipEvent_t ev_parsed = nullptr;
    // after the last fb_flow_history_dev: it reads the last update's shared scratch (history words,
    // partials, slot counts, combined-entry slots), which the next update rewrites -- that update
    // waits for it on every stream it uses, whichever stream the history ran on
    hipEvent_t ev_hist = nullptr;
    bool hist_pending = false;
    hipEvent_t ev_upd[2] = {nullptr, nullptr};  // after the update of async batch k (k & 1)
    uint64_t async_k = 0;                       // async batches issued
    uint32_t* d_rec_part2 = nullptr;            // partitions of the odd async batches
    const void* async_prev[3] = {nullptr, nullptr, nullptr};  // the last async batch's records, counts, stats
    uint32_t upd_word[2] = {4u, 4u};            // error word (launch & 3) of the async update in slot k & 1 (4: none)
    uint32_t* d_agg_slot = nullptr;       // [flow_recs / 2 + 1] table slot per combined entry
    uint32_t last_set = 0;                // the update scratch set of the last update (history)
    // the last update, for fb_flow_history_dev
    const fb_pkt_out* last_recs = nullptr;
    const uint32_t* last_part = nullptr;  // the fused parse's per-record words of the last update
    const uint32_t* last_seg = nullptr;
    const fb_batch_stats* last_stats = nullptr;
    uint32_t last_slots = 0;
    uint32_t last_chunks = 0;
    FlowParams last_p;                    // the last update's parameters (fb_flow_history_dev)
    uint32_t* d_hcount = nullptr;         // [table_cap] history characters per slot of the last update
    uint32_t* d_part_base = nullptr;      // [flow_parts + 1] history output offset per partition
    uint32_t* d_hist_slow = nullptr;      // [flow_parts + 1] count + partitions for the general history kernel
    uint32_t* d_hist_cnt = nullptr;       // per-block slot counts of hot history partitions (lazy)
    uint64_t hist_cnt_bytes = 0;
    // enrichment tables (fb_set_asn_tables / fb_set_blacklists)
    fb_asn_range* d_asn4 = nullptr;
    fb_asn_range* d_asn6 = nullptr;
    uint32_t n_asn4 = 0, n_asn6 = 0;
    uint32_t* d_bl4_pos = nullptr;
    unsigned long long* d_bl4_mask = nullptr;
    uint4* d_bl6_pos = nullptr;
    unsigned long long* d_bl6_mask = nullptr;
    uint32_t m_bl4 = 0, m_bl6 = 0;
    // host-mode staging
    uint8_t* s_frames = nullptr;
    uint64_t s_frames_cap = 0;
    uint32_t* s_offsets = nullptr;
    fb_pkt_out* s_out = nullptr;
    fb_dns_out* s_dns = nullptr;
    uint8_t* s_cls = nullptr;
    uint64_t s_pkts_cap = 0;
    fb_batch_stats* s_stats = nullptr;
};

int fbk::ctx_device(const fb_ctx* c) { return c->device; }

// A call (or a ring batch) reported a nonzero device error word: the scratch the launches share
// (stats tick words, error words) is zeroed before the context's next launch.
int fbk::ctx_report_error(fb_ctx* c, uint64_t e) {
    c->need_reset = true;
    if (e & 4u) return set_err(FB_ERR_TABLE_FULL, "flow table full (error word %llu)", (unsigned long long)e);
    return set_err(FB_ERR_INTERNAL, "device error word %llu (2: offset scan expired, 8: update scratch "
                   "overflow, 16: table-update spin expired, 32: dense tile offset past the batch)",
                   (unsigned long long)e);
}

// Entry points that read or write the table or the update scratch first order their stream after
// the last pipelined update (fb_process_seg_async_dev runs updates on the context's own stream);
// host code that frees or rewrites that scratch waits for it.
static int join_updates(fb_ctx* c, hipStream_t s) {
    if (c->async_k == 0) return FB_OK;
    HIP_TRY(hipStreamWaitEvent(s, c->ev_upd[(c->async_k - 1u) & 1u], 0));
    return FB_OK;
}
// A parse launch zeroes the error word of the launch after it ((launch + 1) & 3).  A pipelined
// update still in flight may own that word (it sets bits there and copies it into its stats at
// the end): the stream waits for that update first, so no failure bit of it is lost.
static int guard_next_error_word(fb_ctx* c, hipStream_t s) {
    if (c->async_k == 0) return FB_OK;
    const uint32_t z = (c->epoch + 2u) & 3u;
    for (uint32_t k = 0; k < 2; ++k)
        if (c->upd_word[k] == z) HIP_TRY(hipStreamWaitEvent(s, c->ev_upd[k], 0));
    return FB_OK;
}
static int drain_updates(fb_ctx* c) {
    if (c->async_k && c->upd) HIP_TRY(hipStreamSynchronize(c->upd));
    if (c->hist_pending) HIP_TRY(hipEventSynchronize(c->ev_hist));  // (before scratch is freed)
    return FB_OK;
}

namespace fbk {
bool build_blacklist_tables(const fb_cidr* nets, uint32_t n, std::vector<uint32_t>& p4,
                            std::vector<unsigned long long>& m4, std::vector<uint4>& p6,
                            std::vector<unsigned long long>& m6);
}

static EnrichTables enrich_tables(const fb_ctx* c) {
    EnrichTables t;
    t.asn4 = c->d_asn4;
    t.asn6 = c->d_asn6;
    t.n4 = c->n_asn4;
    t.n6 = c->n_asn6;
    t.bl4_pos = c->d_bl4_pos;
    t.bl4_mask = c->d_bl4_mask;
    t.bl6_pos = c->d_bl6_pos;
    t.bl6_mask = c->d_bl6_mask;
    t.m4 = c->m_bl4;
    t.m6 = c->m_bl6;
    return t;
}

// Replace a device array with a copy of host data (n elements); empty -> nullptr.
template <typename T>
static int upload_array(T** d, const T* h, size_t n) {
    if (*d) (void)hipFree(*d);
    *d = nullptr;
    if (n == 0) return FB_OK;
    if (hipMalloc((void**)d, n * sizeof(T)) != hipSuccess) return set_err(FB_ERR_NOMEM, "enrichment table");
    HIP_TRY(hipMemcpy(*d, h, n * sizeof(T), hipMemcpyHostToDevice));
    return FB_OK;
}

static void free_upd_scratch(UpdScratch& u) {
    hipFree(u.entries);
    hipFree(u.comb);
    hipFree(u.rows);
    hipFree(u.cols);
    hipFree(u.rows_h);
    hipFree(u.e_orig);
    hipFree(u.e_sort);
    hipFree(u.hot);
    hipFree(u.ctl);
    hipFree(u.order);
    u = UpdScratch();
}

// One update scratch set sized for c->flow_recs records.
static int alloc_upd_scratch(fb_ctx* c, UpdScratch& u, hipStream_t s) {
    const uint64_t recs = c->flow_recs, chunks = recs / kFlowChunk;
    if (hipMalloc(&u.entries, recs * 4ull) != hipSuccess ||
        hipMalloc(&u.comb, (uint64_t)c->comb_cap * 2ull * sizeof(FlowEntry)) != hipSuccess ||
        hipMalloc(&u.rows_h, chunks * c->flow_parts * 4ull) != hipSuccess ||
        hipMalloc(&u.e_orig, recs * 4ull) != hipSuccess || hipMalloc(&u.e_sort, recs * 8ull) != hipSuccess ||
        hipMalloc(&u.rows, chunks * c->flow_parts * 4ull) != hipSuccess ||
        hipMalloc(&u.cols, chunks * c->flow_parts * 4ull) != hipSuccess ||
        hipMalloc(&u.hot, (recs / 16 + 16) * 4ull) != hipSuccess || hipMalloc(&u.ctl, 16) != hipSuccess ||
        hipMalloc(&u.order, ((uint64_t)c->flow_parts + kK2Lead + 1u) * 4ull) != hipSuccess) {
        free_upd_scratch(u);
        return set_err(FB_ERR_NOMEM, "flow update scratch (%llu records)", (unsigned long long)recs);
    }
    HIP_TRY(hipMemsetAsync(u.ctl, 0, 16, s));
    return FB_OK;
}

// Session-table update scratch for batches of up to `recs` records (grown, never shrunk).
static int ensure_flow_scratch(fb_ctx* c, uint64_t recs, hipStream_t s) {
    if (!c->d_table) return FB_OK;
    recs = std::max<uint64_t>(recs, kFlowChunk);
    recs = (recs + kFlowChunk - 1) / kFlowChunk * kFlowChunk;
    if (recs <= c->flow_recs) return FB_OK;
    int rc = drain_updates(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    const bool had_set1 = c->us[1].entries != nullptr;
    for (UpdScratch& u : c->us) free_upd_scratch(u);
    hipFree(c->d_hword);
    hipFree(c->d_rec_part);
    hipFree(c->d_rec_part2);
    hipFree(c->d_rec_ent);
    hipFree(c->d_rec_ent2);
    hipFree(c->d_agg_slot);
    c->d_rec_part = c->d_rec_part2 = nullptr;
    c->d_rec_ent = c->d_rec_ent2 = nullptr;
    c->part_recs = nullptr;
    c->part_buf = nullptr;
    c->ent_buf = nullptr;
    c->d_hword = nullptr;
    c->comb_cap = 0;
    c->d_agg_slot = nullptr;
    c->last_recs = nullptr;  // its scratch is gone
    c->last_part = nullptr;
    c->flow_recs = 0;
    if (hipMalloc(&c->d_hword, recs * 4ull) != hipSuccess || hipMalloc(&c->d_rec_part, recs * 4ull) != hipSuccess ||
        hipMalloc(&c->d_rec_ent, recs * 16ull * kUpdEntU4) != hipSuccess ||
        hipMalloc(&c->d_agg_slot, (recs / 2 + 1) * 4ull) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "flow update scratch (%llu records)", (unsigned long long)recs);
    c->flow_recs = recs;
    // combined entries: at most one per two records of the hot groups; a quarter of the batch's
    // records is room for any skew we measured (past it a hot group just stays plain)
    c->comb_cap = (uint32_t)(recs / 4 + 256);
    rc = alloc_upd_scratch(c, c->us[0], s);
    if (!rc && had_set1) rc = alloc_upd_scratch(c, c->us[1], s);
    return rc;
}

static int empty_update(fb_ctx* c);

static int upload_cfg(fb_ctx* c, hipStream_t s) {
    if (!c->cfg_dirty) return FB_OK;
    HIP_TRY(hipStreamSynchronize(s));  // nothing on this stream may still read d_cfg
    HIP_TRY(hipMemcpyAsync(c->d_cfg, c->h_cfg, sizeof(DevConfig), hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->cfg_dirty = false;
    return FB_OK;
}

// Zero the stats tick words and both error words before the next launch (at create, and after
// a call reported an error).  Stream-ordered: the launches run on `s`, which may be a
// non-blocking stream that does not synchronise with the null stream.
static int reset_launch_scratch(fb_ctx* c, hipStream_t s) {
    if (!c->need_reset) return FB_OK;
    const int rc = drain_updates(c);  // a pipelined update may still write an error word
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_tick, 0, kTickWords * 8ull, s));
    HIP_TRY(hipMemsetAsync(c->d_error, 0, 16, s));
    c->need_reset = false;
    return FB_OK;
}

static uint64_t dense_status_words(uint64_t nseg) { return nseg / parse_dense_tile_segs() + 1; }

// Scan scratch of the dense entry points, for batches of up to `n` frames (grown, never shrunk).
static int ensure_compact_scratch(fb_ctx* c, uint64_t n, hipStream_t s) {
    const uint64_t nseg = (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
    if (nseg <= c->cseg_cap) return FB_OK;
    HIP_TRY(hipStreamSynchronize(s));
    hipFree(c->d_cseg);
    hipFree(c->d_cpre);
    hipFree(c->d_cstatus);
    hipFree(c->d_cticket);
    hipFree(c->d_dstatus);
    c->d_cseg = nullptr;
    c->d_cpre = nullptr;
    c->d_cstatus = nullptr;
    c->d_cticket = nullptr;
    c->d_dstatus = nullptr;
    c->cseg_cap = 0;
    c->scan_epoch = 0;
    c->dense_epoch = 0;
    const uint64_t want = std::max<uint64_t>(nseg, 1024);
    if (hipMalloc(&c->d_cseg, want * 4ull) != hipSuccess || hipMalloc(&c->d_cpre, want * 8ull) != hipSuccess ||
        hipMalloc(&c->d_cstatus, seg_scan_tiles((uint32_t)want) * 8ull) != hipSuccess ||
        hipMalloc(&c->d_cticket, 4) != hipSuccess ||
        hipMalloc(&c->d_dstatus, dense_status_words(want) * 8ull) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "dense-output scratch (%llu segments)", (unsigned long long)want);
    HIP_TRY(hipMemsetAsync(c->d_cticket, 0, 4, s));
    c->cseg_cap = want;
    return FB_OK;
}

// The next scan's scratch: a fresh epoch (the status words are zeroed, stream-ordered, when the
// 8-bit epoch wraps).
static int scan_scratch(fb_ctx* c, hipStream_t s, SegScanScratch& sc) {
    if (c->scan_epoch == 0u || c->scan_epoch >= 255u) {
        HIP_TRY(hipMemsetAsync(c->d_cstatus, 0, seg_scan_tiles((uint32_t)c->cseg_cap) * 8ull, s));
        c->scan_epoch = 0u;
    }
    sc.status = c->d_cstatus;
    sc.ticket = c->d_cticket;
    sc.epoch = ++c->scan_epoch;
    sc.err = c->d_error + (c->epoch & 3u);
    return FB_OK;
}

static void set_lan(DevConfig* d, const fb_lan_v6* nets, uint32_t n) {
    d->n_lan_v6 = n;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t p = std::min<uint32_t>(nets[i].prefix, 128u);
        for (int k = 0; k < 4; ++k) {
            int bits = (int)p - 32 * k;
            uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : 0xFFFFFFFFu << (32 - bits));
            d->lan_v6[i].mask[k] = m;
            d->lan_v6[i].net[k] = nets[i].net[k] & m;
        }
    }
}

extern "C" {

uint32_t fb_abi_version(void) { return FB_ABI_VERSION; }
const char* fb_last_error(void) { return g_err; }

int fb_device_count(int* n) {
    if (!n) return set_err(FB_ERR_INVAL, "n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = e == hipSuccess ? c : 0;
    return FB_OK;
}

int fb_ctx_device(const fb_ctx* ctx, int* device) {
    if (!ctx || !device) return set_err(FB_ERR_INVAL, "ctx or device is NULL");
    *device = ctx->device;
    return FB_OK;
}

fb_ctx* fb_create(int device, const fb_config* cfg) {
    if (!cfg) { set_err(FB_ERR_INVAL, "cfg is NULL"); return nullptr; }
    if (cfg->abi_version != FB_ABI_VERSION) {
        set_err(FB_ERR_INVAL, "abi_version %u != %u", cfg->abi_version, FB_ABI_VERSION);
        return nullptr;
    }
    if (cfg->filter > FB_FILTER_ALL || cfg->n_lan_v6 > FB_MAX_LAN_V6 || cfg->n_own_ips > FB_MAX_OWN_IPS ||
        (cfg->n_lan_v6 && !cfg->lan_v6) || (cfg->n_own_ips && !cfg->own_ips)) {
        set_err(FB_ERR_INVAL, "invalid fb_config field");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        set_err(FB_ERR_NODEV, "device %d not available (%d HIP devices)", device, ndev);
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_err(FB_ERR_NODEV, "device %d is not gfx950 (%s)", device, prop.gcnArchName);
        return nullptr;
    }
    DeviceGuard g(device);
    fb_ctx* c = new (std::nothrow) fb_ctx();
    if (!c) { set_err(FB_ERR_NOMEM, "fb_ctx"); return nullptr; }
    c->device = device;
    {
        // The segmented kernel streams with no inter-workgroup wait; its grid is the co-resident
        // block count only so that every block stays busy until the batch is done.
        int sb = 0;
        if (occupancy_parse_seg(&sb) != hipSuccess || sb < 1) sb = 1;
        c->seg_grid = std::min<uint32_t>((uint32_t)(sb * prop.multiProcessorCount), 1023u);  // 10-bit stats tickets
#ifndef FB_ASYNC_BPC
#define FB_ASYNC_BPC 1  // round 3: with unsorted update entries 2 blocks per CU led (12.88 vs 12.55 Gpps);
                        // with the entries sorted by partition 1 block leaves K2 more of each CU
                        // (14.19-14.22 vs 13.74-13.75; 3 blocks 13.49-13.80)
#endif
        c->seg_grid_async = std::min<uint32_t>((uint32_t)(FB_ASYNC_BPC * prop.multiProcessorCount), c->seg_grid);
        int db = 0;
        if (occupancy_parse_dense(&db) != hipSuccess || db < 1) db = 1;
        c->dense_grid = std::min<uint32_t>((uint32_t)(db * prop.multiProcessorCount), 1023u);  // 10-bit stats tickets
    }
    c->h_cfg = new (std::nothrow) DevConfig();
    bool ok = c->h_cfg != nullptr;
    if (ok) {
        memset(c->h_cfg, 0, sizeof(DevConfig));
        memcpy(c->h_cfg->service_bitmap, cfg->service_bitmap ? cfg->service_bitmap : kDefaultServiceBitmap,
               FB_SERVICE_BITMAP_BYTES);
        c->h_cfg->filter = cfg->filter;
        set_lan(c->h_cfg, cfg->lan_v6, cfg->n_lan_v6);
        c->h_cfg->n_own = cfg->n_own_ips;
        for (uint32_t i = 0; i < cfg->n_own_ips; ++i) c->h_cfg->own[i] = cfg->own_ips[i];
    }
    ok = ok && hipMalloc(&c->d_cfg, sizeof(DevConfig)) == hipSuccess;
    ok = ok && hipMalloc(&c->d_error, 16) == hipSuccess && hipMemset(c->d_error, 0, 16) == hipSuccess;
    ok = ok && hipMalloc(&c->d_tick, kTickWords * 8ull) == hipSuccess &&
         hipMemset(c->d_tick, 0, kTickWords * 8ull) == hipSuccess;
    ok = ok && hipMalloc(&c->d_n, 16) == hipSuccess;
    if (ok && cfg->flow_capacity > kFlowMaxCapacity) {
        set_err(FB_ERR_INVAL, "flow_capacity %llu > %llu slots", (unsigned long long)cfg->flow_capacity,
                (unsigned long long)kFlowMaxCapacity);
        ok = false;
    }
    if (ok && cfg->flow_capacity) {
        uint64_t cap = kFlowSlots;
        while (cap < cfg->flow_capacity) cap <<= 1;
        c->table_cap = cap;
        c->flow_parts = (uint32_t)(cap / kFlowSlots);
        uint32_t lg = 0;
        while ((1u << lg) < c->flow_parts) ++lg;
        c->flow_shift = 64u - lg;
        ok = hipMalloc(&c->d_table, cap * sizeof(FlowSlot)) == hipSuccess &&
             hipMemset(c->d_table, 0, cap * sizeof(FlowSlot)) == hipSuccess &&
             hipMalloc(&c->d_char_call, cap * sizeof(uint4)) == hipSuccess &&
             hipMalloc(&c->d_partials, 4ull * c->flow_parts * 8ull) == hipSuccess &&
             hipMalloc(&c->d_hcount, cap * 4ull) == hipSuccess &&
             hipMalloc(&c->d_part_base, (c->flow_parts + 1ull) * 4ull) == hipSuccess &&
             hipMalloc(&c->d_hist_slow, (c->flow_parts + 1ull) * 4ull) == hipSuccess &&
             hipHostMalloc((void**)&c->h_mbox, sizeof(FlowMailbox), hipHostMallocMapped) == hipSuccess &&
             hipHostGetDevicePointer((void**)&c->d_mbox, c->h_mbox, 0) == hipSuccess;
        if (ok) memset(c->h_mbox, 0, sizeof(FlowMailbox));
        c->grow = (cfg->flags & FB_CFG_FIXED_TABLE) == 0u;
        c->timed = (cfg->flags & FB_CFG_TIMED) != 0u;
        if (ok && c->timed)
            ok = hipMalloc(&c->d_time, cap * sizeof(FlowTime)) == hipSuccess &&
                 hipMemset(c->d_time, 0, cap * sizeof(FlowTime)) == hipSuccess &&
                 hipEventCreateWithFlags(&c->ev_tscratch, hipEventDisableTiming) == hipSuccess;
        ok = ok && ensure_flow_scratch(c, cfg->max_batch_packets, nullptr) == FB_OK;
    }
    ok = ok && upload_cfg(c, nullptr) == FB_OK;
    if (!ok) {
        if (g_err[0] == 0) set_err(FB_ERR_NOMEM, "device allocation failed");
        fb_destroy(c);
        return nullptr;
    }
    return c;
}

int fb_destroy(fb_ctx* c) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    DeviceGuard g(c->device);
    (void)hipDeviceSynchronize();
    hipFree(c->d_cfg);
    hipFree(c->d_tick);
    hipFree(c->d_cseg);
    hipFree(c->d_cpre);
    hipFree(c->d_cstatus);
    hipFree(c->d_cticket);
    hipFree(c->d_dstatus);
    hipFree(c->d_error);
    hipFree(c->d_table);
    for (UpdScratch& u : c->us) free_upd_scratch(u);
    hipFree(c->d_partials);
    hipFree(c->d_remap);
    hipFree(c->d_char_call);
    hipFree(c->d_time);
    hipFree(c->d_tscratch);
    if (c->ev_tscratch) hipEventDestroy(c->ev_tscratch);
    hipFree(c->d_mscratch);
    if (c->ev_mscratch) hipEventDestroy(c->ev_mscratch);
    if (c->h_mbox) hipHostFree(c->h_mbox);
    hipFree(c->d_n);
    hipFree(c->d_hword);
    hipFree(c->d_rec_part);
    hipFree(c->d_rec_part2);
    hipFree(c->d_rec_ent);
    hipFree(c->d_rec_ent2);
    hipFree(c->d_agg_slot);
    if (c->upd) hipStreamDestroy(c->upd);
    if (c->ev_parsed) hipEventDestroy(c->ev_parsed);
    if (c->ev_hist) hipEventDestroy(c->ev_hist);
    for (hipEvent_t e : c->ev_upd)
        if (e) hipEventDestroy(e);
    hipFree(c->d_asn4);
    hipFree(c->d_asn6);
    hipFree(c->d_bl4_pos);
    hipFree(c->d_bl4_mask);
    hipFree(c->d_bl6_pos);
    hipFree(c->d_bl6_mask);
    hipFree(c->d_hcount);
    hipFree(c->d_part_base);
    hipFree(c->d_hist_slow);
    hipFree(c->d_hist_cnt);
    hipFree(c->s_frames);
    hipFree(c->s_offsets);
    hipFree(c->s_out);
    hipFree(c->s_dns);
    hipFree(c->s_cls);
    hipFree(c->s_stats);
    delete c->h_cfg;
    delete c;
    return FB_OK;
}

int fb_set_filter(fb_ctx* c, uint32_t filter) {
    if (!c || filter > FB_FILTER_ALL) return set_err(FB_ERR_INVAL, "bad ctx or filter");
    if (c->h_cfg->filter != filter) { c->h_cfg->filter = filter; c->cfg_dirty = true; }
    return FB_OK;
}

int fb_set_service_bitmap(fb_ctx* c, const uint8_t* bm) {
    if (!c || !bm) return set_err(FB_ERR_INVAL, "bad ctx or bitmap");
    memcpy(c->h_cfg->service_bitmap, bm, FB_SERVICE_BITMAP_BYTES);
    c->cfg_dirty = true;
    return FB_OK;
}

int fb_set_lan_v6(fb_ctx* c, const fb_lan_v6* nets, uint32_t n) {
    if (!c || n > FB_MAX_LAN_V6 || (n && !nets)) return set_err(FB_ERR_INVAL, "bad lan_v6 table");
    set_lan(c->h_cfg, nets, n);
    c->cfg_dirty = true;
    return FB_OK;
}

int fb_set_stage_event(fb_ctx* c, void* event) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    c->stage_event = (hipEvent_t)event;  // the caller's event (fb_event_create); not owned
    return FB_OK;
}

int fb_set_frame_times(fb_ctx* c, const uint64_t* d_ts) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (!c->timed) return set_err(FB_ERR_INVAL, "the context was created without FB_CFG_TIMED");
    c->next_ts = reinterpret_cast<const unsigned long long*>(d_ts);
    return FB_OK;
}

// Every update call of a timed context consumes the frame times set before it (checked before the
// call's parse, so a refused call changes nothing).
static int timed_ready(fb_ctx* c) {
    if (c->timed && !c->next_ts)
        return set_err(FB_ERR_INVAL, "a timed context needs fb_set_frame_times before each update call");
    return FB_OK;
}

int fb_debug_set(fb_ctx* c, uint32_t knob, uint64_t value) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    switch (knob) {
        case FB_DEBUG_DENSE_STEAL_POLLS:
            c->steal_polls = (uint32_t)std::min<uint64_t>(value, 0xFFFFFFFFull);
            return FB_OK;
        case FB_DEBUG_DENSE_OFFSET_SKEW:
            if (value > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "skew %llu >= 2^32", (unsigned long long)value);
            c->dn_skew = value;
            if (value) fprintf(stderr, "flodbadd_gpu: FB_DEBUG_DENSE_OFFSET_SKEW %llu active on this context (fault injection)\n",
                               (unsigned long long)value);
            return FB_OK;
        default:
            return set_err(FB_ERR_INVAL, "unknown debug knob %u", knob);
    }
}

int fb_set_session_records(fb_ctx* c, int emit) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    c->emit_records = emit != 0;
    return FB_OK;
}

int fb_set_own_ips(fb_ctx* c, const fb_ip* ips, uint32_t n) {
    if (!c || n > FB_MAX_OWN_IPS || (n && !ips)) return set_err(FB_ERR_INVAL, "bad own-ip table");
    c->h_cfg->n_own = n;
    for (uint32_t i = 0; i < n; ++i) c->h_cfg->own[i] = ips[i];
    c->cfg_dirty = true;
    return FB_OK;
}

// Launch of the segmented streaming kernel over `sb` (frames, or the parsed packets `parsed`).
// `want_parts`: one frame batch whose session table update follows (fb_process_seg_dev) -- the
// kernel also writes each SESSION record slot's table partition, so the update's histogram pass
// reads 4 B per record instead of the record.
#ifdef FB_SEG_TRACE
static unsigned long long* g_strace = nullptr;
// diagnostic builds only: the last k_parse_seg launch's per-block trace (4 x 2048 words), after a sync
extern "C" __attribute__((visibility("default"))) int fb_seg_trace_last(unsigned long long* out) {
    if (!g_strace || hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpy(out, g_strace, 8u * 4u * 2048u, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
static int launch_seg(fb_ctx* c, const SegBatches& sb, uint32_t n_max, const fb_parsed_pkt* parsed, hipStream_t s,
                      bool want_parts = false, SegPass pass = SegPass::kSegments, fb_pkt_out* dense_out = nullptr,
                      fb_dns_out* dense_dns = nullptr) {
    int rc = reset_launch_scratch(c, s);
    // a fused parse rewrites d_rec_part, which a pipelined update may still read (the pipelined
    // call itself writes its own slot's buffer and orders that wait itself)
    if (!rc && want_parts && !c->part_target) rc = join_updates(c, s);
    if (!rc) rc = upload_cfg(c, s);
    if (!rc) rc = ensure_flow_scratch(c, n_max, s);
    if (rc) return rc;
    c->last_n = n_max;
    ParseParams p;
    memset(&p, 0, sizeof(p));
    p.pre = c->d_cpre;
    p.dense_out = dense_out;
    p.dense_dns = dense_dns;
    p.parsed = parsed;
    p.n = parsed ? sb.b[0].n : 0u;
    p.rec_part = (want_parts && sb.count == 1u && c->d_table) ? (c->part_target ? c->part_target : c->d_rec_part)
                                                              : nullptr;
    p.rec_ent = p.rec_part ? (c->ent_target ? c->ent_target : c->d_rec_ent) : nullptr;
    p.no_records = p.rec_part && !c->emit_records ? 1u : 0u;
    p.part_shift = c->flow_shift;
    c->part_recs = p.rec_part ? sb.b[0].out : nullptr;
    c->part_buf = p.rec_part;
    c->ent_buf = p.rec_ent;
    p.cfg = c->d_cfg;
    p.tick = c->d_tick;
    if (pass != SegPass::kDenseOut) {
        rc = guard_next_error_word(c, s);
        if (rc) return rc;
    }
    // dense pass 2 belongs to pass 1's launch: same error word, no new parity
    const uint32_t launch = pass == SegPass::kDenseOut ? c->epoch : ++c->epoch;
    p.error = c->d_error + (launch & 3u);
    p.error_next = c->d_error + ((launch + 1u) & 3u);
    const uint32_t waves = parse_seg_block_threads() / 64u;
    const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>(c->seg_grid, (sb.total_segs + waves - 1) / waves));
#ifdef FB_SEG_TRACE
    if (!g_strace && hipMalloc(&g_strace, 8u * 4u * 2048u) != hipSuccess) return set_err(FB_ERR_NOMEM, "trace");
    HIP_TRY(hipMemsetAsync(g_strace, 0, 8u * 4u * 2048u, s));
    p.dtrace = g_strace;
#endif
    HIP_TRY(launch_parse_seg(p, sb, grid, s, pass));
    return FB_OK;
}

static SegBatches one_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets, uint32_t n,
                            fb_pkt_out* out, uint32_t* seg, uint8_t* cls, fb_batch_stats* stats) {
    SegBatches sb;
    memset(&sb, 0, sizeof(sb));
    sb.count = 1;
    SegBatch& B = sb.b[0];
    B.frames = frames;
    B.offsets = offsets;
    B.out = out;
    B.seg = seg;
    B.cls = cls;
    B.stats = stats;
    B.n = n;
    B.frames_bytes = (uint32_t)frames_bytes;
    sb.total_segs = (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
    return sb;
}

int fb_parse_classify_seg_batches_dev(fb_ctx* c, const fb_seg_batch* batches, uint32_t count, void* stream) {
    if (!c || !batches || count == 0 || count > FB_MAX_SEG_BATCHES)
        return set_err(FB_ERR_INVAL, "ctx, batches and 1 <= count <= FB_MAX_SEG_BATCHES are required");
    SegBatches sb;
    memset(&sb, 0, sizeof(sb));
    uint64_t segs = 0;
    uint32_t n_max = 0;
    for (uint32_t k = 0; k < count; ++k) {
        const fb_seg_batch& x = batches[k];
        if (!x.d_stats) return set_err(FB_ERR_INVAL, "batch %u: d_stats is required", k);
        if (x.n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "batch %u: n > FB_MAX_BATCH_PACKETS", k);
        if (x.frames_bytes > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "batch %u: frames_bytes must be < 4 GiB", k);
        if (!x.d_offsets || (x.n && (!x.d_out || !x.d_seg)))
            return set_err(FB_ERR_INVAL, "batch %u: d_offsets, d_out and d_seg are required", k);
        if (x.n && x.frames_bytes && !x.d_frames) return set_err(FB_ERR_INVAL, "batch %u: d_frames is NULL", k);
        SegBatch& B = sb.b[k];
        B.frames = x.d_frames;
        B.offsets = x.d_offsets;
        B.out = x.d_out;
        B.seg = x.d_seg;
        B.cls = x.d_class;
        B.stats = x.d_stats;
        B.n = x.n;
        B.frames_bytes = (uint32_t)x.frames_bytes;
        B.seg_start = (uint32_t)segs;
        segs += (x.n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
        n_max = std::max(n_max, x.n);
    }
    if (segs > 0xFFFFFFFFull / FB_SEG_FRAMES) return set_err(FB_ERR_INVAL, "too many frames in one launch");
    sb.count = count;
    sb.total_segs = (uint32_t)segs;
    DeviceGuard g(c->device);
    return launch_seg(c, sb, n_max, nullptr, (hipStream_t)stream);
}

#ifdef FB_DN_TRACE
static unsigned long long* g_dtrace = nullptr;
// diagnostic builds only: the last dense launch's trace (4 x (8192 + 1024) words), after a device sync
extern "C" __attribute__((visibility("default"))) int fb_dense_trace_last(unsigned long long* out) {
    if (!g_dtrace || hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpy(out, g_dtrace, 8u * 4u * (8192u + 1024u), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
// ---- resident queue-fed parse (k_parse_seg_queue, fb_parse.hip) ------------------------------------
#ifdef FB_QUEUE_TRACE
static unsigned long long g_qtrace[kQTraceAll];
#endif
struct fb_seg_queue {
    int device = 0;
    uint32_t depth = 0;  // batches in flight at most
    uint32_t slots = 0;  // ring slots: depth rounded up to a power of two (the kernel masks)
    hipStream_t stream = nullptr;
    QueueHost* h = nullptr;      // pinned, coherent host memory (the kernel's ring and completion words)
    QueueHost* h_dev = nullptr;  // its device alias
    QueueDev* d_ring = nullptr;  // the device side of the ring
    DevConfig* d_cfg = nullptr;  // the context's configuration when the queue was created
    unsigned long long* d_tick = nullptr;
    uint32_t* d_blk = nullptr;
    uint32_t* d_head = nullptr;
    uint32_t* d_err = nullptr;
    unsigned long long* d_trace = nullptr;  // -DFB_QUEUE_TRACE builds
    uint64_t submitted = 0;
    uint64_t limit = FB_QUEUE_MAX_SUBMISSIONS;  // the kernel's batch numbers are 32-bit (k_parse_seg_queue)
    bool launched = false;
    hipError_t gone = hipSuccess;  // what the stream reported when the kernel was found gone
    uint32_t grid = 0;             // the kernel's blocks (all must be resident at once)
    uint64_t idle_ns = 0;          // idle_ms in ns
    std::chrono::steady_clock::time_point created;
    bool not_resident = false;     // its blocks were not all running idle_ms after create
    bool counted = false;          // holds its device's live-queue count
};
// One live queue per device: a second one's blocks could never all be resident beside the first's
// (two blocks per CU each), so its kernel would not start and nothing on the device could report it.
static std::mutex g_queue_mu;
static uint32_t g_queue_live[64];

static void queue_free(fb_seg_queue* q) {
    if (q->counted) {
        std::lock_guard<std::mutex> lk(g_queue_mu);
        --g_queue_live[q->device];
    }
    if (q->stream) hipStreamDestroy(q->stream);
    hipFree(q->d_cfg);
    hipFree(q->d_tick);
    hipFree(q->d_blk);
    hipFree(q->d_head);
    hipFree(q->d_err);
    hipFree(q->d_ring);
    hipFree(q->d_trace);
    if (q->h) hipHostFree(q->h);
    delete q;
}

static uint64_t hload(const unsigned long long* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

// FB_OK once the kernel is gone or going (a block expired, or -- every `every` calls, a runtime call --
// the kernel has ended), 1 while it runs
static int queue_kernel_gone(fb_seg_queue* q, uint64_t spin, uint64_t every) {
    if (hload(&q->h->status) & kQueueExpired) return FB_OK;
    if (spin % every != every - 1u) return 1;
    const hipError_t e = hipStreamQuery(q->stream);
    if (e == hipErrorNotReady) {
        // every block counts itself into pad[3] when it starts; a kernel some of whose blocks never
        // ran (the CUs held by other work) cannot complete a batch, and its resident blocks are not
        // the ones waiting -- only the host can notice
        if (hload(&q->h->pad[3]) != q->grid &&
            (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                          q->created).count() > q->idle_ns) {
            q->not_resident = true;
            return FB_OK;
        }
        return 1;
    }
    q->gone = e;
    return FB_OK;
}

static int queue_gone_error(fb_seg_queue* q) {
    const QueueHost* h = q->h;
    if (q->not_resident)
        return set_err(FB_ERR_INTERNAL,
                       "the queue kernel's blocks are not all running (%llu of %u started within idle_ms): the "
                       "device's CUs are held by other work; destroy the queue",
                       (unsigned long long)hload(&h->pad[3]), q->grid);
    return set_err(FB_ERR_INTERNAL,
                   "the queue kernel has stopped (status %llu, stream: %s; a block left after %llu ticks idle "
                   "waiting for batch %llu (block %llu), tail %llu): destroy the queue",
                   (unsigned long long)hload(&h->status), hipGetErrorString(q->gone), (unsigned long long)hload(&h->pad[0]),
                   (unsigned long long)(hload(&h->pad[1]) & 0xFFFFFFFFu), (unsigned long long)(hload(&h->pad[1]) >> 32),
                   (unsigned long long)hload(&h->pad[2]));
}

fb_seg_queue* fb_seg_queue_create(fb_ctx* c, uint32_t depth, uint32_t idle_ms) {
    return fb_seg_queue_create_ex(c, depth, idle_ms, 0u);
}

fb_seg_queue* fb_seg_queue_create_ex(fb_ctx* c, uint32_t depth, uint32_t idle_ms, uint32_t flags) {
    if (flags & ~FB_QUEUE_SHARED) {
        set_err(FB_ERR_INVAL, "unknown queue flags 0x%x", flags);
        return nullptr;
    }
    if (!c) {
        set_err(FB_ERR_INVAL, "ctx is NULL");
        return nullptr;
    }
    if (depth == 0u) depth = 8u;
    if (depth > kQueueMax) {
        set_err(FB_ERR_INVAL, "depth %u > FB_QUEUE_MAX_DEPTH", depth);
        return nullptr;
    }
    DeviceGuard g(c->device);
    {
        std::lock_guard<std::mutex> lk(g_queue_mu);
        if (c->device < 0 || c->device >= 64) {
            set_err(FB_ERR_INVAL, "device %d", c->device);
            return nullptr;
        }
        if (g_queue_live[c->device]) {
            set_err(FB_ERR_INVAL, "device %d already runs a queue (one per device: destroy it first)", c->device);
            return nullptr;
        }
        ++g_queue_live[c->device];  // (released by queue_free, or below)
    }
    fb_seg_queue* q = new (std::nothrow) fb_seg_queue();
    if (!q) {
        std::lock_guard<std::mutex> lk(g_queue_mu);
        --g_queue_live[c->device];
        set_err(FB_ERR_NOMEM, "queue");
        return nullptr;
    }
    q->counted = true;
    q->device = c->device;
    q->depth = depth;
    q->slots = 1u;
    while (q->slots < depth) q->slots <<= 1;
    bool ok = hipHostMalloc((void**)&q->h, sizeof(QueueHost), hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
    if (ok) {
        memset(q->h, 0, sizeof(QueueHost));
        ok = hipHostGetDevicePointer((void**)&q->h_dev, q->h, 0) == hipSuccess;
    }
    ok = ok && hipMalloc(&q->d_cfg, sizeof(DevConfig)) == hipSuccess &&
         hipMemcpy(q->d_cfg, c->h_cfg, sizeof(DevConfig), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMalloc(&q->d_tick, kQueueMax * 8u * 8u) == hipSuccess && hipMemset(q->d_tick, 0, kQueueMax * 64u) == hipSuccess;
    ok = ok && hipMalloc(&q->d_blk, kQueueMax * 4u) == hipSuccess && hipMemset(q->d_blk, 0, kQueueMax * 4u) == hipSuccess;
    ok = ok && hipMalloc(&q->d_head, kQueueMax * kQueueHeadWords * 4u) == hipSuccess &&
         hipMemset(q->d_head, 0, kQueueMax * kQueueHeadWords * 4u) == hipSuccess;
    ok = ok && hipMalloc(&q->d_err, 4) == hipSuccess && hipMemset(q->d_err, 0, 4) == hipSuccess;
    ok = ok && hipMalloc(&q->d_ring, sizeof(QueueDev)) == hipSuccess && hipMemset(q->d_ring, 0, sizeof(QueueDev)) == hipSuccess;
    ok = ok && hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking) == hipSuccess;
#ifdef FB_QUEUE_TRACE
    if (ok) {
        std::vector<unsigned long long> t0((size_t)kQTraceAll, 0ull);
        std::fill(t0.begin() + kQtFirst * kQTraceN, t0.begin() + (kQtArr0 + 1) * kQTraceN, ~0ull);
        ok = hipMalloc(&q->d_trace, t0.size() * 8u) == hipSuccess &&
             hipMemcpy(q->d_trace, t0.data(), t0.size() * 8u, hipMemcpyHostToDevice) == hipSuccess;
    }
#endif
    if (!ok) {
        queue_free(q);
        set_err(FB_ERR_NOMEM, "queue resources");
        return nullptr;
    }
    QueueParams p;
    p.cfg = q->d_cfg;
    p.h = q->h_dev;
    p.d = q->d_ring;
    p.tick = q->d_tick;
    p.blk_done = q->d_blk;
    p.head = q->d_head;
    p.error = q->d_err;
    p.depth = q->slots;
    p.idle_ticks = (unsigned long long)(idle_ms ? idle_ms : 5000u) * 100000ull;  // s_memrealtime: 100 MHz
    p.trace = q->d_trace;
    // two blocks per CU, not k_parse_seg's three: the resident kernel must leave room on every CU for
    // the work the host issues while it runs -- blit kernels of pageable copies (a capture loop reads
    // its results back), other streams' kernels; at three blocks (80 VGPRs x 6 waves per SIMD) a D2H
    // copy into pageable memory waited until the queue's kernel had left (round-5 probe)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus < 1) cus = 1;
    // every block must be resident at once: a batch completes when every block has passed it
    int occ = 0;
    if (occupancy_parse_seg_queue(&occ) != hipSuccess || occ < 1) occ = 1;
    // FB_QUEUE_SHARED: one block per CU, so the session-table update kernels (K1 96 KB + K2 80 KB of
    // LDS, 80 / 128 VGPRs) fit beside it (two blocks leave ~66 KB of LDS)
    const int bpc = (flags & FB_QUEUE_SHARED) ? 1 : FB_QUEUE_BPC;
    uint32_t grid = std::min<uint32_t>(c->seg_grid, (uint32_t)(std::min(bpc, occ) * cus));
    // ... and on only a share of the CUs (the dispatcher spreads a small grid one block per CU): K2's
    // two 80-KB workgroups per CU need a CU's whole LDS, so every CU holding a queue block runs one.
    // C4-mix 1M-frame batches + the update beside them: CUs / 1, 2, 4, 8, 16, 32 -> 1.8, 2.6, 3.3,
    // 3.75, 2.3, 1.2 Gpps (past 8 the parse on too few CUs is the step; profiles/r06_shared_queue_div_sweep.txt)
    if (flags & FB_QUEUE_SHARED) grid = std::max<uint32_t>(1u, grid / FB_QUEUE_SHARED_DIV);
    q->grid = grid;
    q->idle_ns = (uint64_t)(idle_ms ? idle_ms : 5000u) * 1000000ull;
    q->created = std::chrono::steady_clock::now();
    if (launch_parse_seg_queue(p, grid, q->stream) != hipSuccess) {
        queue_free(q);
        set_err(FB_ERR_HIP, "queue kernel launch");
        return nullptr;
    }
    q->launched = true;
    return q;
}

int fb_seg_queue_submit(fb_seg_queue* q, const fb_seg_batch* x, uint64_t* ticket) {
    if (!q || !x) return set_err(FB_ERR_INVAL, "queue and batch are required");
    if (!x->d_stats) return set_err(FB_ERR_INVAL, "d_stats is required");
    if (x->n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n > FB_MAX_BATCH_PACKETS");
    if (x->frames_bytes > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "frames_bytes must be < 4 GiB");
    if (!x->d_offsets || (x->n && (!x->d_out || !x->d_seg))) return set_err(FB_ERR_INVAL, "d_offsets, d_out and d_seg are required");
    if (x->n && x->frames_bytes && !x->d_frames) return set_err(FB_ERR_INVAL, "d_frames is NULL");
    const uint64_t k = q->submitted, S = q->slots;
    // the kernel carries batch numbers, ring claims and completion words in 32 bits: past 2^32 a
    // claim's expected value and a slot's completion word would repeat an old batch's, so a queue
    // takes at most `limit` batches and is then recycled by the host
    if (k >= q->limit)
        return set_err(FB_ERR_INVAL, "the queue took its %llu batches (32-bit batch numbers): destroy it and create a "
                       "new one", (unsigned long long)q->limit);
    // at most `depth` batches in flight, and a slot is reused only once its previous batch (k - S) is
    // complete -- its completion word is stored after the kernel has reset the slot's state
    const uint64_t back[2] = {q->depth, S};
    for (const uint64_t b : back) {
        if (k < b) continue;  // (no such batch yet)
        const uint64_t prev = k - b;
        for (uint64_t spin = 0; hload(&q->h->cdone[prev & (S - 1u)]) != prev + 1u; ++spin) {
            if (queue_kernel_gone(q, spin, 4096u) == FB_OK && hload(&q->h->cdone[prev & (S - 1u)]) != prev + 1u)
                return queue_gone_error(q);
            __builtin_ia32_pause();
        }
    }
    QueueHost* h = q->h;
    memcpy((void*)&h->desc[k & (S - 1u)], x, sizeof(fb_seg_batch));
    __atomic_store_n(&h->tail, (unsigned long long)(k + 1u), __ATOMIC_RELEASE);  // after the descriptor
    q->submitted = k + 1u;
    if (ticket) *ticket = k;
    return FB_OK;
}

int fb_seg_queue_set_limit(fb_seg_queue* q, uint64_t limit) {
    if (!q) return set_err(FB_ERR_INVAL, "queue is NULL");
    if (limit > FB_QUEUE_MAX_SUBMISSIONS || limit < q->submitted)
        return set_err(FB_ERR_INVAL, "limit %llu outside [%llu, FB_QUEUE_MAX_SUBMISSIONS]", (unsigned long long)limit,
                       (unsigned long long)q->submitted);
    q->limit = limit;
    return FB_OK;
}

static int queue_poll(fb_seg_queue* q, uint64_t t, uint64_t spin, uint64_t every) {
    if (!q) return set_err(FB_ERR_INVAL, "queue is NULL");
    if (t >= q->submitted) return set_err(FB_ERR_INVAL, "ticket %llu was not issued", (unsigned long long)t);
    if (t + q->depth < q->submitted) return FB_OK;  // a later submission waited for it
    const uint64_t slot = t & (q->slots - 1u);
    if (hload(&q->h->cdone[slot]) == t + 1u) return FB_OK;
    if (queue_kernel_gone(q, spin, every) == FB_OK && hload(&q->h->cdone[slot]) != t + 1u)
        return queue_gone_error(q);
    return 1;
}

int fb_seg_queue_query(fb_seg_queue* q, uint64_t t) { return queue_poll(q, t, 0u, 1u); }

int fb_seg_queue_wait(fb_seg_queue* q, uint64_t t) {
    for (uint64_t spin = 0;; ++spin) {
        const int rc = queue_poll(q, t, spin, 4096u);
        if (rc != 1) return rc;
        __builtin_ia32_pause();
    }
}

int fb_seg_queue_destroy(fb_seg_queue* q) {
    if (!q) return set_err(FB_ERR_INVAL, "queue is NULL");
    DeviceGuard g(q->device);
    __atomic_store_n(&q->h->stop, 1ull, __ATOMIC_RELEASE);  // the kernel leaves once the submitted batches are done
    int rc = FB_OK;
    if (q->launched && hipStreamSynchronize(q->stream) != hipSuccess) rc = set_err(FB_ERR_HIP, "queue kernel");
#ifdef FB_QUEUE_TRACE
    if (q->d_trace) hipMemcpy(g_qtrace, q->d_trace, sizeof(g_qtrace), hipMemcpyDeviceToHost);
#endif
    queue_free(q);
    return rc;
}
#ifdef FB_QUEUE_TRACE
// diagnostic builds only: the last destroyed queue's trace (kQTraceAll words: QTrace order, then per block)
extern "C" __attribute__((visibility("default"))) int fb_seg_queue_trace_last(unsigned long long* out) {
    memcpy(out, g_qtrace, sizeof(g_qtrace));
    return (int)kQTraceAll;
}
#endif

static int parse_seg(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets, uint32_t n,
                     fb_pkt_out* d_out, uint32_t* d_seg, uint8_t* d_class, fb_batch_stats* d_stats, void* stream,
                     bool want_parts) {
    if (!c || !d_stats) return set_err(FB_ERR_INVAL, "ctx and d_stats are required");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (frames_bytes > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "frames_bytes must be < 4 GiB");
    if (n && (!d_offsets || !d_out || !d_seg)) return set_err(FB_ERR_INVAL, "d_offsets, d_out and d_seg are required");
    if (n && frames_bytes && !d_frames) return set_err(FB_ERR_INVAL, "d_frames is NULL");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_stats, 0, sizeof(fb_batch_stats), s));
        return FB_OK;
    }
    return launch_seg(c, one_batch(d_frames, frames_bytes, d_offsets, n, d_out, d_seg, d_class, d_stats), n, nullptr,
                      s, want_parts);
}

int fb_parse_classify_seg_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                              uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg, uint8_t* d_class,
                              fb_batch_stats* d_stats, void* stream) {
    return parse_seg(c, d_frames, frames_bytes, d_offsets, n, d_out, d_seg, d_class, d_stats, stream, false);
}

int fb_process_parsed_seg_dev(fb_ctx* c, const fb_parsed_pkt* d_in, uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg,
                              uint8_t* d_class, fb_batch_stats* d_stats, void* stream) {
    if (!c || !d_stats) return set_err(FB_ERR_INVAL, "ctx and d_stats are required");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (n && (!d_in || !d_out || !d_seg)) return set_err(FB_ERR_INVAL, "d_in, d_out and d_seg are required");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_stats, 0, sizeof(fb_batch_stats), s));
        return FB_OK;
    }
    return launch_seg(c, one_batch(nullptr, 0, nullptr, n, d_out, d_seg, d_class, d_stats), n, d_in, s);
}

int fb_seg_compact_dev(fb_ctx* c, const fb_pkt_out* d_seg_out, const uint32_t* d_seg, uint32_t n, fb_pkt_out* d_out,
                       fb_dns_out* d_dns, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (n && (!d_seg_out || !d_seg)) return set_err(FB_ERR_INVAL, "d_seg_out and d_seg are required");
    if (n == 0 || (!d_out && !d_dns)) return FB_OK;
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_compact_scratch(c, n, s);
    if (rc) return rc;
    SegScanScratch sc;
    rc = scan_scratch(c, s, sc);
    if (rc) return rc;
    HIP_TRY(launch_seg_compact(d_seg_out, d_seg, (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES, c->d_cpre, sc, d_out, d_dns,
                               s));
    return FB_OK;
}

// Dense output in two passes of the segmented kernel (fb_compact.hip): pass 1 counts every 64-frame
// segment (classes and batch stats too), the scan turns the counts into batch-wide offsets, pass 2
// parses again and stores each record at its offset -- at C2 the frames are still in the Infinity
// Cache for pass 2.  No kernel of the path waits on another workgroup.
// Frame batches take the single-pass kernel (k_parse_dense: tiles ordered by ticket, decoupled
// look-back, records kept in registers until the tile's offset is known); parsed-packet batches
// (and FB_DENSE_TWO_PASS builds, for A/B timing) the two passes below.
static int parse_dense_single(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                              uint32_t n, fb_pkt_out* d_out, fb_dns_out* d_dns, uint8_t* d_class,
                              fb_batch_stats* d_stats, hipStream_t s) {
    int rc = reset_launch_scratch(c, s);
    if (!rc) rc = upload_cfg(c, s);
    if (!rc) rc = ensure_flow_scratch(c, n, s);
    if (!rc) rc = ensure_compact_scratch(c, n, s);
    if (rc) return rc;
    const uint32_t nseg = (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
    if (c->dense_epoch == 0u || c->dense_epoch >= 255u) {
        HIP_TRY(hipMemsetAsync(c->d_dstatus, 0, dense_status_words(c->cseg_cap) * 8ull, s));
        c->dense_epoch = 0u;
    }
    c->last_n = n;
    c->part_recs = nullptr;
    c->part_buf = nullptr;
    ParseParams p;
    memset(&p, 0, sizeof(p));
    p.cfg = c->d_cfg;
    p.tick = c->d_tick;
    rc = guard_next_error_word(c, s);
    if (rc) return rc;
    const uint32_t launch = ++c->epoch;
    p.error = c->d_error + (launch & 3u);
    p.error_next = c->d_error + ((launch + 1u) & 3u);
    p.dense_out = d_out;
    p.dense_dns = d_dns;
    p.dstatus = c->d_dstatus;
    p.steal_polls = c->steal_polls;
    p.dn_skew = c->dn_skew;
#ifdef FB_DN_TRACE
    if (!g_dtrace) {
        if (hipMalloc(&g_dtrace, 8u * 4u * (8192u + 1024u)) != hipSuccess) return set_err(FB_ERR_NOMEM, "trace");
    }
    HIP_TRY(hipMemsetAsync(g_dtrace, 0, 8u * 4u * (8192u + 1024u), s));
    p.dtrace = g_dtrace;
#endif
    p.dep = ++c->dense_epoch;
    p.ntiles = (nseg + parse_dense_tile_segs() - 1) / parse_dense_tile_segs();
    const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>(c->dense_grid, p.ntiles));
    SegBatch b;
    memset(&b, 0, sizeof(b));
    b.frames = d_frames;
    b.offsets = d_offsets;
    b.cls = d_class;
    b.stats = d_stats;
    b.n = n;
    b.frames_bytes = (uint32_t)frames_bytes;
    HIP_TRY(launch_parse_dense(p, b, grid, s));
    return FB_OK;
}

static int parse_dense(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                       const fb_parsed_pkt* d_in, uint32_t n, fb_pkt_out* d_out, fb_dns_out* d_dns, uint8_t* d_class,
                       fb_batch_stats* d_stats, hipStream_t s) {
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_stats, 0, sizeof(fb_batch_stats), s));
        return FB_OK;
    }
#ifndef FB_DENSE_TWO_PASS
    if (!d_in) return parse_dense_single(c, d_frames, frames_bytes, d_offsets, n, d_out, d_dns, d_class, d_stats, s);
#endif
    int rc = ensure_compact_scratch(c, n, s);
    if (rc) return rc;
    rc = launch_seg(c, one_batch(d_frames, frames_bytes, d_offsets, n, nullptr, c->d_cseg, d_class, d_stats), n, d_in,
                    s, false, SegPass::kCount);
    if (rc || (!d_out && !d_dns)) return rc;
    const uint32_t nseg = (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
    SegScanScratch sc;
    rc = scan_scratch(c, s, sc);
    if (rc) return rc;
    HIP_TRY(launch_seg_scan(c->d_cseg, nseg, c->d_cpre, sc, s));
    return launch_seg(c, one_batch(d_frames, frames_bytes, d_offsets, n, nullptr, nullptr, nullptr, nullptr), n, d_in, s,
                      false, SegPass::kDenseOut, d_out, d_dns);
}

int fb_parse_classify_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes,
                          const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out, fb_dns_out* d_dns,
                          uint8_t* d_class, fb_batch_stats* d_stats, void* stream) {
    if (!c || !d_stats) return set_err(FB_ERR_INVAL, "ctx and d_stats are required");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (frames_bytes > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "frames_bytes must be < 4 GiB");
    if (n && !d_offsets) return set_err(FB_ERR_INVAL, "d_offsets is NULL");
    if (n && frames_bytes && !d_frames) return set_err(FB_ERR_INVAL, "d_frames is NULL");
    DeviceGuard g(c->device);
    return parse_dense(c, d_frames, frames_bytes, d_offsets, nullptr, n, d_out, d_dns, d_class, d_stats,
                       (hipStream_t)stream);
}

int fb_process_parsed_dev(fb_ctx* c, const fb_parsed_pkt* d_in, uint32_t n, fb_pkt_out* d_out,
                          uint8_t* d_class, fb_batch_stats* d_stats, void* stream) {
    if (!c || !d_stats) return set_err(FB_ERR_INVAL, "ctx and d_stats are required");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (n && !d_in) return set_err(FB_ERR_INVAL, "d_in is NULL");
    DeviceGuard g(c->device);
    return parse_dense(c, nullptr, 0, nullptr, d_in, n, d_out, nullptr, d_class, d_stats, (hipStream_t)stream);
}

static int ensure_staging(fb_ctx* c, uint64_t n, uint64_t bytes) {
    if (bytes > c->s_frames_cap) {
        hipFree(c->s_frames);
        c->s_frames = nullptr;
        c->s_frames_cap = 0;
        uint64_t want = std::max<uint64_t>(bytes, 1 << 20);
        if (hipMalloc(&c->s_frames, want) != hipSuccess) return set_err(FB_ERR_NOMEM, "staging frames");
        c->s_frames_cap = want;
    }
    if (n > c->s_pkts_cap) {
        hipFree(c->s_offsets); hipFree(c->s_out); hipFree(c->s_dns); hipFree(c->s_cls);
        c->s_offsets = nullptr; c->s_out = nullptr; c->s_dns = nullptr; c->s_cls = nullptr;
        c->s_pkts_cap = 0;
        uint64_t want = std::max<uint64_t>(n, 4096);
        if (hipMalloc(&c->s_offsets, (want + 1) * 4) != hipSuccess ||
            hipMalloc(&c->s_out, want * sizeof(fb_pkt_out)) != hipSuccess ||
            hipMalloc(&c->s_dns, want * sizeof(fb_dns_out)) != hipSuccess ||
            hipMalloc(&c->s_cls, want) != hipSuccess)
            return set_err(FB_ERR_NOMEM, "staging packets");
        c->s_pkts_cap = want;
    }
    if (!c->s_stats && hipMalloc(&c->s_stats, sizeof(fb_batch_stats)) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "staging stats");
    return FB_OK;
}

static int check_error_word(fb_ctx* c, hipStream_t s) {
    uint32_t e = 0;
    HIP_TRY(hipMemcpyAsync(&e, c->d_error + (c->epoch & 3u), 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (e) return ctx_report_error(c, e);
    return FB_OK;
}

int fb_parse_classify(fb_ctx* c, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                      uint32_t n, fb_pkt_out* out, uint32_t* n_out, fb_dns_out* dns, uint32_t* n_dns,
                      uint8_t* cls, fb_batch_stats* stats, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n too large");
    if (frames_bytes > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "frames_bytes must be < 4 GiB");
    if ((n && !offsets) || (frames_bytes && !frames)) return set_err(FB_ERR_INVAL, "NULL input");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_staging(c, n, frames_bytes);
    if (rc) return rc;
    if (frames_bytes) HIP_TRY(hipMemcpyAsync(c->s_frames, frames, frames_bytes, hipMemcpyHostToDevice, s));
    if (n) HIP_TRY(hipMemcpyAsync(c->s_offsets, offsets, (uint64_t)(n + 1) * 4, hipMemcpyHostToDevice, s));
    rc = fb_parse_classify_dev(c, c->s_frames, frames_bytes, c->s_offsets, n, out ? c->s_out : nullptr,
                               dns ? c->s_dns : nullptr, cls ? c->s_cls : nullptr, c->s_stats, s);
    if (rc) return rc;
    fb_batch_stats st;
    HIP_TRY(hipMemcpyAsync(&st, c->s_stats, sizeof(st), hipMemcpyDeviceToHost, s));
    rc = check_error_word(c, s);  // synchronises the stream
    if (rc) return rc;
    if (out && st.n_session)
        HIP_TRY(hipMemcpyAsync(out, c->s_out, st.n_session * sizeof(fb_pkt_out), hipMemcpyDeviceToHost, s));
    if (dns && st.n_dns)
        HIP_TRY(hipMemcpyAsync(dns, c->s_dns, st.n_dns * sizeof(fb_dns_out), hipMemcpyDeviceToHost, s));
    if (cls && n) HIP_TRY(hipMemcpyAsync(cls, c->s_cls, n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (n_out) *n_out = (uint32_t)st.n_session;
    if (n_dns) *n_dns = (uint32_t)st.n_dns;
    if (stats) *stats = st;
    return FB_OK;
}

int fb_process_parsed(fb_ctx* c, const fb_parsed_pkt* in, uint32_t n, fb_pkt_out* out, uint32_t* n_out,
                      uint8_t* cls, fb_batch_stats* stats, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n too large");
    if (n && !in) return set_err(FB_ERR_INVAL, "NULL input");
    if (c->d_table) {
        if (int rc = timed_ready(c)) return rc;
    }
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_staging(c, n, (uint64_t)n * sizeof(fb_parsed_pkt));
    if (rc) return rc;
    const fb_parsed_pkt* d_in = reinterpret_cast<const fb_parsed_pkt*>(c->s_frames);
    if (n) HIP_TRY(hipMemcpyAsync(c->s_frames, in, (uint64_t)n * sizeof(fb_parsed_pkt), hipMemcpyHostToDevice, s));
    rc = fb_process_parsed_dev(c, d_in, n, c->s_out, cls ? c->s_cls : nullptr, c->s_stats, s);
    if (rc) return rc;
    if (n && c->d_table) {
        rc = fb_flow_update_dev(c, c->s_out, c->s_stats, s);
        if (rc) return rc;
    } else if (c->d_table) {
        empty_update(c);
    }
    fb_batch_stats st;
    HIP_TRY(hipMemcpyAsync(&st, c->s_stats, sizeof(st), hipMemcpyDeviceToHost, s));
    rc = check_error_word(c, s);  // synchronises the stream
    if (rc) return rc;
    if (out && st.n_session)
        HIP_TRY(hipMemcpyAsync(out, c->s_out, st.n_session * sizeof(fb_pkt_out), hipMemcpyDeviceToHost, s));
    if (cls && n) HIP_TRY(hipMemcpyAsync(cls, c->s_cls, n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (n_out) *n_out = (uint32_t)st.n_session;
    if (stats) *stats = st;
    return FB_OK;
}

// An update call without records still counts as one (the high word of flow positions).
static int empty_update(fb_ctx* c) {
    ++c->flow_batch;
    c->next_ts = nullptr;
    c->last_recs = nullptr;
    c->last_part = nullptr;
    return FB_OK;
}

// ---- table growth -------------------------------------------------------------------------------
// Doubles the table on the device: every slot re-inserted into 2x partitions (k_flow_grow), the old
// -> new slot map kept for fb_flow_slot_remap.  Drains the updates in flight first: growth is rare.
static int grow_table(fb_ctx* c, hipStream_t s, uint32_t k) {
    int rc = drain_updates(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t cap = c->table_cap << k;
    FlowSlot* nw = nullptr;
    unsigned long long* partials = nullptr;
    if (hipMalloc(&nw, cap * sizeof(FlowSlot)) != hipSuccess) return set_err(FB_ERR_NOMEM, "grown flow table");
    uint32_t *hcount = nullptr, *part_base = nullptr, *hist_slow = nullptr;
    auto free_new = [&]() {
        hipFree(partials);
        hipFree(hcount);
        hipFree(part_base);
        hipFree(hist_slow);
    };
    if (hipMalloc(&partials, 4ull * (cap / kFlowSlots) * 8ull) != hipSuccess ||
        hipMalloc(&hcount, cap * 4ull) != hipSuccess ||
        hipMalloc(&part_base, (cap / kFlowSlots + 1ull) * 4ull) != hipSuccess ||
        hipMalloc(&hist_slow, (cap / kFlowSlots + 1ull) * 4ull) != hipSuccess) {
        free_new();
        hipFree(nw);
        return set_err(FB_ERR_NOMEM, "grown flow table partials");
    }
    hipFree(c->d_remap);
    c->d_remap = nullptr;
    c->remap_n = 0;
    if (hipMalloc(&c->d_remap, c->table_cap * 4ull) != hipSuccess) {
        hipFree(nw);
        free_new();
        return set_err(FB_ERR_NOMEM, "slot remap");
    }
    HIP_TRY(hipMemsetAsync(nw, 0, cap * sizeof(FlowSlot), s));
    uint4* nw_cc = nullptr;
    if (hipMalloc(&nw_cc, cap * sizeof(uint4)) != hipSuccess) {
        hipFree(nw);
        free_new();
        return set_err(FB_ERR_NOMEM, "grown character-call array");
    }
    HIP_TRY(launch_flow_grow(c->d_table, c->flow_parts, k, c->flow_shift - k, nw, c->d_remap, c->d_char_call, nw_cc,
                             s));
    FlowTime* nw_time = nullptr;
    if (c->timed) {  // the time records follow their flows' new slots
        if (hipMalloc(&nw_time, cap * sizeof(FlowTime)) != hipSuccess) {
            hipFree(nw);
            hipFree(nw_cc);
            free_new();
            return set_err(FB_ERR_NOMEM, "grown time plane");
        }
        HIP_TRY(hipMemsetAsync(nw_time, 0, cap * sizeof(FlowTime), s));
        HIP_TRY(launch_time_remap(c->d_time, c->d_remap, c->table_cap, nw_time, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (c->timed) {
        hipFree(c->d_time);
        c->d_time = nw_time;
    }
    hipFree(c->d_table);
    hipFree(c->d_partials);
    hipFree(c->d_hcount);
    hipFree(c->d_part_base);
    hipFree(c->d_hist_slow);
    c->d_table = nw;
    hipFree(c->d_char_call);
    c->d_char_call = nw_cc;
    c->d_partials = partials;
    c->d_hcount = hcount;
    c->d_part_base = part_base;
    c->d_hist_slow = hist_slow;
    c->remap_n = c->table_cap;
    c->table_cap = cap;
    c->flow_parts <<= k;
    c->flow_shift -= k;
    c->grown_seq = c->upd_seq;
    ++c->generation;
    // scratch sized by the partition count (K1 rows / K2 columns), history sort bits: rebuilt
    const uint64_t recs = c->flow_recs;
    const bool had_set1 = c->us[1].entries != nullptr;
    for (UpdScratch& u : c->us) free_upd_scratch(u);
    c->flow_recs = 0;
    rc = ensure_flow_scratch(c, recs, s);
    if (!rc && had_set1) rc = alloc_upd_scratch(c, c->us[1], s);
    c->last_recs = nullptr;  // the last update's slots moved: its history is no longer available
    c->last_part = nullptr;
    return rc;
}

// Before an update call: grow while the occupancy the last completed update reported, plus the new
// flows of the updates still in flight (each estimated at the last reported update's count) and of
// this one (twice that: arrival rates rise), spread over the partitions, plus slack for the spread
// between partitions, would pass 7/8 of a partition, or the flows 3/4 of the table.  The report sits
// in host-mapped memory; the decision needs the report of the update two calls back (the second call
// after a create / clear: the first update's), so a host that enqueues asynchronous batches faster
// than the device runs them waits here for that report (the device keeps the previous batch's work)
// instead of projecting from an older one -- or from none, which let the table fill.  A burst
// beyond the estimate inside one batch can still fill a partition: the update then reports error
// bit 4 (FB_ERR_TABLE_FULL).
static constexpr uint64_t kGrowPart = kFlowSlots * 7u / 8u;
static constexpr double kMailboxWaitS = 120.0;
static int maybe_grow(fb_ctx* c, hipStream_t s) {
    if (!c->d_table || !c->grow || c->part_recs) return FB_OK;  // (a fused parse already bucketed for this geometry)
    const volatile FlowMailbox* m = c->h_mbox;
    const uint64_t issued = c->upd_seq - c->clear_seq;              // updates since create / clear
    const uint64_t need = c->clear_seq + (issued >= 2u ? issued - 1u : issued);
    uint64_t seq = __atomic_load_n(&m->seq, __ATOMIC_ACQUIRE);
    if (seq < need) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0; (seq = __atomic_load_n(&m->seq, __ATOMIC_ACQUIRE)) < need; ++spin) {
            if (spin > 64u) std::this_thread::yield();
            if ((spin & 1023u) == 0u &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kMailboxWaitS)
                return set_err(FB_ERR_HIP, "no table-occupancy report from update %llu after %.0f s",
                               (unsigned long long)need, kMailboxWaitS);
        }
    }
    if (seq == 0 || seq <= c->clear_seq) return FB_OK;
    const uint64_t flows = m->flows, newf = m->new_flows;
    const uint64_t ahead = c->upd_seq - seq + 2u;  // in flight, plus this call counted twice
    // the smallest k (table x 2^k) that holds the projection: one growth (one slot remap) per call
    uint32_t k = 0;
    for (;; ++k) {
        const uint64_t parts = (uint64_t)c->flow_parts << k;
        if ((c->table_cap << k) > kFlowMaxCapacity || k > 5u) {
            if (k > 0) --k;
            break;
        }
        // a report from before a growth describes other partitions: only its flow count is used there
        const uint64_t maxp = (k == 0 && seq > c->grown_seq) ? m->max_part : flows / parts + 3u * kFlowSlots / 16u;
        const uint64_t add = (ahead * newf + parts - 1u) / parts;
        if (maxp + add + kFlowSlots / 32u <= kGrowPart && flows + ahead * newf <= (c->table_cap << k) * 3u / 4u) break;
    }
    return k ? grow_table(c, s, k) : FB_OK;
}

// One table update.  `split` (the pipelined call): the bucketing kernels (K1, K1c) run on `s_bucket`
// -- the caller's stream (possibly the null stream), right after the parse that wrote the batch's
// partitions, into update scratch set `set` -- and the rest (K1t, K2, the stats fold) on `s` after
// an event; otherwise everything runs on `s` with set 0.
static int flow_update(fb_ctx* c, const fb_pkt_out* d_recs, const uint32_t* d_seg, uint32_t n_slots,
                       fb_batch_stats* d_stats, hipStream_t s, bool split = false, hipStream_t s_bucket = nullptr,
                       uint32_t set = 0) {
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    DeviceGuard g(c->device);
    if (!split) s_bucket = s;
    int rc = split ? FB_OK : join_updates(c, s);
    if (!rc && !split) rc = maybe_grow(c, s);  // (skipped after a fused parse: it bucketed for this geometry)
    if (!rc) rc = ensure_flow_scratch(c, n_slots, s_bucket);
    if (!rc && set == 1u && !c->us[1].entries) rc = alloc_upd_scratch(c, c->us[1], s_bucket);
    if (rc) return rc;
    if (c->hist_pending) {  // the last history's reads of the shared update scratch come first
        HIP_TRY(hipStreamWaitEvent(s_bucket, c->ev_hist, 0));
        if (s != s_bucket) HIP_TRY(hipStreamWaitEvent(s, c->ev_hist, 0));
        c->hist_pending = false;
    }
    const UpdScratch& u = c->us[set];
    // record slots of the batch: at most last_n records (dense) / n_slots slots (segmented)
    const uint32_t chunks = (uint32_t)std::max<uint64_t>(1, ((uint64_t)n_slots + kFlowChunk - 1) / kFlowChunk);
    FlowParams p;
    p.recs = d_recs;
    p.seg = d_seg;
    p.n_slots = n_slots;
    p.stats = d_stats;
    p.table = c->d_table;
    p.entries = u.entries;
    p.comb = u.comb;
    p.comb_cap = c->comb_cap;
    p.rows = u.rows;
    p.cols = u.cols;
    p.partials = c->d_partials;
    p.error = c->d_error + (c->epoch & 3u);
    p.max_recs = (uint32_t)std::min<uint64_t>((uint64_t)chunks * kFlowChunk, c->flow_recs);
    p.parts = c->flow_parts;
    p.part_shift = c->flow_shift;
    p.chunk_stride = (uint32_t)(c->flow_recs / kFlowChunk);
    p.batch = c->flow_batch;
    p.rows_h = u.rows_h;
    p.e_orig = u.e_orig;
    p.e_sort = u.e_sort;
    p.hcount = c->d_hcount;
    p.part_base = c->d_part_base;
    p.hword = c->d_hword;
    p.hot = u.hot;
    p.ctl = u.ctl;
#ifndef FB_K2_ORDER
#define FB_K2_ORDER 1
#endif
    p.order = FB_K2_ORDER ? u.order : nullptr;
    p.agg_slot = c->d_agg_slot;
    p.hot_cap = (uint32_t)(c->flow_recs / 16 + 16);
    p.rec_part = (d_seg && c->part_recs == d_recs) ? c->part_buf : nullptr;  // written by this batch's parse
    p.ent = p.rec_part ? c->ent_buf : nullptr;                                  // (with its update entries)
    p.char_call = c->d_char_call;
    c->part_recs = nullptr;
    if (c->timed) {  // the capture-time pass's scratch (K2 writes its sort input into it)
        const uint32_t slots = p.max_recs < n_slots ? p.max_recs : n_slots;
        uint32_t bits = 0;
        while ((1ull << bits) < c->table_cap) ++bits;
        const uint64_t need = time_scratch_bytes(slots, bits);
        HIP_TRY(hipStreamWaitEvent(s, c->ev_tscratch, 0));
        if (need > c->tscratch_bytes) {
            HIP_TRY(hipEventSynchronize(c->ev_tscratch));
            hipFree(c->d_tscratch);
            c->d_tscratch = nullptr;
            c->tscratch_bytes = 0;
            if (hipMalloc(&c->d_tscratch, need) != hipSuccess)
                return set_err(FB_ERR_NOMEM, "capture-time scratch (%llu bytes)", (unsigned long long)need);
            c->tscratch_bytes = need;
        }
        p.tkv = time_key_array(c->d_tscratch);
        HIP_TRY(launch_time_prepare(c->d_tscratch, slots, s));
        p.hot = nullptr;  // no combined entries: every record is a plain entry K2 places
    }
    HIP_TRY(launch_flow_bucket(p, chunks, s_bucket));
    if (split) {
        // (K1t stays on the update stream: beside the next batch's parse it takes ~95 us instead of
        // 10, but on the parse stream it delays that parse instead -- C4 12.85 vs 12.57 Gpps)
        HIP_TRY(hipEventRecord(c->ev_parsed, s_bucket));
        HIP_TRY(hipStreamWaitEvent(s, c->ev_parsed, 0));
    }
    HIP_TRY(launch_flow_apply(p, chunks, s));
    HIP_TRY(launch_flow_finish(d_stats, c->d_partials, c->flow_parts, c->d_error + (c->epoch & 3u), c->d_mbox,
                               ++c->upd_seq, s));
    if (c->timed) {  // the capture-time pass over the placed records (fb_time.hip)
        const uint32_t slots = p.max_recs < n_slots ? p.max_recs : n_slots;
        HIP_TRY(launch_time_update(p, slots, c->table_cap, c->d_time, c->next_ts, c->d_tscratch, s));
        HIP_TRY(hipEventRecord(c->ev_tscratch, s));
        c->next_ts = nullptr;
    }
    ++c->flow_batch;
    c->last_set = set;
    c->last_recs = d_recs;
    c->last_part = p.rec_part;
    c->last_seg = d_seg;
    c->last_stats = d_stats;
    c->last_slots = p.max_recs < n_slots ? p.max_recs : n_slots;
    c->last_chunks = chunks;
    c->last_p = p;
    return FB_OK;
}

int fb_flow_update_dev(fb_ctx* c, const fb_pkt_out* d_recs, fb_batch_stats* d_stats, void* stream) {
    if (!c || !d_recs || !d_stats) return set_err(FB_ERR_INVAL, "ctx, d_recs and d_stats are required");
    if (int rc = timed_ready(c)) return rc;
    return flow_update(c, d_recs, nullptr, c->last_n, d_stats, (hipStream_t)stream);
}

int fb_flow_update_records_dev(fb_ctx* c, const fb_pkt_out* d_recs, uint32_t max_n, fb_batch_stats* d_stats,
                               void* stream) {
    if (!c || !d_stats || (max_n && !d_recs)) return set_err(FB_ERR_INVAL, "ctx, d_recs and d_stats are required");
    if (max_n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "max_n %u > FB_MAX_BATCH_PACKETS", max_n);
    if (int rc = timed_ready(c)) return rc;
    if (max_n == 0) return empty_update(c);
    return flow_update(c, d_recs, nullptr, max_n, d_stats, (hipStream_t)stream);
}

int fb_flow_update_seg_dev(fb_ctx* c, const fb_pkt_out* d_out, const uint32_t* d_seg, uint32_t n,
                           fb_batch_stats* d_stats, void* stream) {
    if (!c || !d_out || !d_seg || !d_stats) return set_err(FB_ERR_INVAL, "ctx, d_out, d_seg and d_stats are required");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (int rc = timed_ready(c)) return rc;
    if (n == 0) return empty_update(c);
    const uint32_t slots = (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES * FB_SEG_FRAMES;
    return flow_update(c, d_out, d_seg, slots, d_stats, (hipStream_t)stream);
}

int fb_process_seg_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                       uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg, uint8_t* d_class, fb_batch_stats* d_stats,
                       void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    int rc = timed_ready(c);
    if (rc) return rc;
    {
        DeviceGuard g(c->device);
        rc = maybe_grow(c, (hipStream_t)stream);  // before the parse writes partitions of this geometry
    }
    if (!rc) rc = parse_seg(c, d_frames, frames_bytes, d_offsets, n, d_out, d_seg, d_class, d_stats, stream, true);
    if (rc == FB_OK && c->stage_event) rc = hipEventRecord(c->stage_event, (hipStream_t)stream) == hipSuccess
                                                ? FB_OK : set_err(FB_ERR_HIP, "stage event record failed");
    if (rc == FB_OK) rc = n == 0 ? empty_update(c) : fb_flow_update_seg_dev(c, d_out, d_seg, n, d_stats, stream);
    c->part_recs = nullptr;  // the partitions serve this update only
    return rc;
}

// Pipelined fb_process_seg_dev: the parse of batch k runs on `stream`, its table update on the
// context's update stream after it, and `stream` waits only for the update of batch k-2 (which
// read the partition buffer and the records this call's slot reuses) -- so the parse of one batch
// overlaps the update of the one before.  Async batch k writes partition buffer k & 1.
int fb_process_seg_async_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                             uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg, uint8_t* d_class,
                             fb_batch_stats* d_stats, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    if (n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "n %u > FB_MAX_BATCH_PACKETS", n);
    if (int rc = timed_ready(c)) return rc;
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    if (!c->upd) {
        if (hipStreamCreateWithFlags(&c->upd, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_parsed, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_upd[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_upd[1], hipEventDisableTiming) != hipSuccess)
            return set_err(FB_ERR_HIP, "update stream / events");
    }
    const uint32_t slot = (uint32_t)(c->async_k & 1u);
    int rc = maybe_grow(c, s);  // before this batch's parse writes partitions (drains the pipeline if it grows)
    if (!rc) rc = ensure_flow_scratch(c, (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES * FB_SEG_FRAMES, s);
    if (rc) return rc;
    if (!c->d_rec_part2 && hipMalloc(&c->d_rec_part2, c->flow_recs * 4ull) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "second partition buffer");
    if (!c->d_rec_ent2 && hipMalloc(&c->d_rec_ent2, c->flow_recs * 16ull * kUpdEntU4) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "second update-entry buffer");
    // the same slot's previous batch (k-2): its update must be done before this parse rewrites the
    // slot's partition buffer; before any async batch, the last synchronous update is on `s` already
    if (c->async_k >= 2) HIP_TRY(hipStreamWaitEvent(s, c->ev_upd[slot], 0));
    // a batch that reuses the previous batch's records, counts or stats buffer waits for its
    // update too (no overlap: rotate two buffer sets to get it)
    if (c->async_k >= 1 && (d_out == c->async_prev[0] || d_seg == c->async_prev[1] || d_stats == c->async_prev[2]))
        HIP_TRY(hipStreamWaitEvent(s, c->ev_upd[slot ^ 1u], 0));
    c->part_target = slot ? c->d_rec_part2 : c->d_rec_part;
    c->ent_target = slot ? c->d_rec_ent2 : c->d_rec_ent;
    const uint32_t grid_full = c->seg_grid;
    c->seg_grid = c->seg_grid_async;
    rc = parse_seg(c, d_frames, frames_bytes, d_offsets, n, d_out, d_seg, d_class, d_stats, stream, true);
    c->seg_grid = grid_full;
    c->part_target = nullptr;
    c->ent_target = nullptr;
    if (rc == FB_OK && c->stage_event) rc = hipEventRecord(c->stage_event, s) == hipSuccess
                                                ? FB_OK : set_err(FB_ERR_HIP, "stage event record failed");
    if (rc) return rc;
    // the bucketing kernels follow the parse on `stream` (into scratch set k & 1, which update k-2
    // -- waited for above -- was the last to read); the update stream takes over after them
    rc = n == 0 ? empty_update(c)
                : flow_update(c, d_out, d_seg, (n + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES * FB_SEG_FRAMES, d_stats,
                              c->upd, true, s, slot);
    c->part_recs = nullptr;
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev_upd[slot], c->upd));
    c->upd_word[slot] = c->epoch & 3u;  // the word flow_update handed this update
    c->async_prev[0] = d_out;
    c->async_prev[1] = d_seg;
    c->async_prev[2] = d_stats;
    ++c->async_k;
    return FB_OK;
}

int fb_flow_join(fb_ctx* c, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    DeviceGuard g(c->device);
    return join_updates(c, (hipStream_t)stream);
}

int fb_process_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const uint32_t* d_offsets,
                   uint32_t n, fb_pkt_out* d_out, fb_dns_out* d_dns, uint8_t* d_class,
                   fb_batch_stats* d_stats, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    if (!d_out) return set_err(FB_ERR_INVAL, "d_out is required");
    if (int rc = timed_ready(c)) return rc;
    int rc = fb_parse_classify_dev(c, d_frames, frames_bytes, d_offsets, n, d_out, d_dns, d_class, d_stats, stream);
    if (rc) return rc;
    if (c->stage_event) HIP_TRY(hipEventRecord(c->stage_event, (hipStream_t)stream));
    if (n == 0) return empty_update(c);
    return fb_flow_update_dev(c, d_out, d_stats, stream);
}

int fb_flow_history_dev(fb_ctx* c, uint8_t* d_hist, uint32_t* d_hist_slot, uint32_t* d_n_hist, void* stream) {
    if (!c || !d_n_hist) return set_err(FB_ERR_INVAL, "ctx and d_n_hist are required");
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    int jr = join_updates(c, s);
    if (jr) return jr;
    const uint32_t n = c->last_recs ? c->last_slots : 0u;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_n_hist, 0, 4, s));
        return FB_OK;
    }
    if (!d_hist || !d_hist_slot) return set_err(FB_ERR_INVAL, "d_hist and d_hist_slot are required");
    const uint64_t cnt_bytes = flow_history_cnt_bytes(c->last_chunks);
    if (cnt_bytes > c->hist_cnt_bytes) {
        HIP_TRY(hipStreamSynchronize(s));
        hipFree(c->d_hist_cnt);
        c->d_hist_cnt = nullptr;
        c->hist_cnt_bytes = 0;
        if (hipMalloc(&c->d_hist_cnt, cnt_bytes) != hipSuccess)
            return set_err(FB_ERR_NOMEM, "history block counts (%llu bytes)", (unsigned long long)cnt_bytes);
        c->hist_cnt_bytes = cnt_bytes;
    }
    if (!c->ev_hist && hipEventCreateWithFlags(&c->ev_hist, hipEventDisableTiming) != hipSuccess)
        return set_err(FB_ERR_HIP, "history event");
    HIP_TRY(launch_flow_history(c->last_p, c->last_chunks, d_hist_slot, d_hist, d_n_hist, c->d_hist_slow,
                                cnt_bytes ? c->d_hist_cnt : nullptr, s));
    HIP_TRY(hipEventRecord(c->ev_hist, s));
    c->hist_pending = true;
    return FB_OK;
}

// ---- enrichment ----------------------------------------------------------------------------
static bool asn_less(const fb_asn_range& a, const fb_asn_range& b, bool v6) {
    const int nw = v6 ? 4 : 1;
    for (int k = 0; k < nw; ++k)
        if (a.start[k] != b.start[k]) return a.start[k] < b.start[k];
    for (int k = 0; k < nw; ++k)
        if (a.end[k] != b.end[k]) return a.end[k] < b.end[k];
    return false;
}

static bool asn_valid(const fb_asn_range& a, bool v6) {  // start <= end (src/asn_db.rs:111-128)
    const int nw = v6 ? 4 : 1;
    for (int k = 0; k < nw; ++k)
        if (a.start[k] != a.end[k]) return a.start[k] < a.end[k];
    return true;
}

int fb_set_asn_tables(fb_ctx* c, const fb_asn_range* v4, uint32_t n4, const fb_asn_range* v6, uint32_t n6) {
    if (!c || (n4 && !v4) || (n6 && !v6)) return set_err(FB_ERR_INVAL, "bad arguments");
    DeviceGuard g(c->device);
    HIP_TRY(hipDeviceSynchronize());  // no launch may still read the old tables
    // Db::from_tsv: drop start > end, then the stable sort by (start, end) (src/asn_db.rs:111-137)
    std::vector<fb_asn_range> a4, a6;
    for (uint32_t i = 0; i < n4; ++i)
        if (asn_valid(v4[i], false)) a4.push_back(v4[i]);
    for (uint32_t i = 0; i < n6; ++i)
        if (asn_valid(v6[i], true)) a6.push_back(v6[i]);
    std::stable_sort(a4.begin(), a4.end(), [](const fb_asn_range& x, const fb_asn_range& y) { return asn_less(x, y, false); });
    std::stable_sort(a6.begin(), a6.end(), [](const fb_asn_range& x, const fb_asn_range& y) { return asn_less(x, y, true); });
    int rc = upload_array(&c->d_asn4, a4.data(), a4.size());
    if (!rc) rc = upload_array(&c->d_asn6, a6.data(), a6.size());
    c->n_asn4 = rc ? 0 : (uint32_t)a4.size();
    c->n_asn6 = rc ? 0 : (uint32_t)a6.size();
    return rc;
}

int fb_set_blacklists(fb_ctx* c, const fb_cidr* nets, uint32_t n) {
    if (!c || (n && !nets)) return set_err(FB_ERR_INVAL, "bad arguments");
    std::vector<uint32_t> p4;
    std::vector<unsigned long long> m4, m6;
    std::vector<uint4> p6;
    if (!build_blacklist_tables(nets, n, p4, m4, p6, m6))
        return set_err(FB_ERR_INVAL, "blacklist entry with a bad family, prefix or list (< %u)", FB_MAX_BLACKLISTS);
    DeviceGuard g(c->device);
    HIP_TRY(hipDeviceSynchronize());
    int rc = upload_array(&c->d_bl4_pos, p4.data(), p4.size());
    if (!rc) rc = upload_array(&c->d_bl4_mask, m4.data(), m4.size());
    if (!rc) rc = upload_array(&c->d_bl6_pos, p6.data(), p6.size());
    if (!rc) rc = upload_array(&c->d_bl6_mask, m6.data(), m6.size());
    c->m_bl4 = rc ? 0 : (uint32_t)p4.size();
    c->m_bl6 = rc ? 0 : (uint32_t)p6.size();
    return rc;
}

int fb_ip_lookup_dev(fb_ctx* c, const fb_ip* d_ips, uint32_t n, int32_t* d_asn, uint64_t* d_lists, void* stream) {
    if (!c || (n && !d_ips)) return set_err(FB_ERR_INVAL, "bad arguments");
    DeviceGuard g(c->device);
    HIP_TRY(launch_ip_lookup(enrich_tables(c), d_ips, n, d_asn, (unsigned long long*)d_lists, (hipStream_t)stream));
    return FB_OK;
}

int fb_flow_enrich_dev(fb_ctx* c, uint32_t new_only, fb_flow_enrich* d_out, uint64_t cap, uint64_t* d_n,
                       void* stream) {
    if (!c || !d_n || (cap && !d_out)) return set_err(FB_ERR_INVAL, "bad arguments");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(d_n, 0, 8, s));
    if (!c->d_table || (new_only && c->flow_batch == 0)) return FB_OK;
    int rc = join_updates(c, s);
    if (!rc) rc = upload_cfg(c, s);
    if (rc) return rc;
    HIP_TRY(launch_flow_enrich(enrich_tables(c), c->d_cfg, c->d_table, c->table_cap, new_only ? 1u : 0u,
                               c->flow_batch - 1u, d_out, cap, (unsigned long long*)d_n, s));
    return FB_OK;
}

int fb_dns_parse_dev(fb_ctx* c, const uint8_t* d_frames, uint64_t frames_bytes, const fb_dns_out* d_dns, uint32_t n,
                     const fb_batch_stats* d_stats, fb_dns_msg* d_msgs, char* d_names, fb_ip* d_addrs, void* stream) {
    if (!c || (n && (!d_dns || !d_msgs || !d_names || !d_addrs || !d_frames)))
        return set_err(FB_ERR_INVAL, "bad arguments");
    if (reinterpret_cast<uintptr_t>(d_names) & 3u) return set_err(FB_ERR_INVAL, "d_names must be 4-byte aligned");
    DeviceGuard g(c->device);
    HIP_TRY(launch_dns_parse(d_frames, frames_bytes, d_dns, n, d_stats, d_msgs, d_names, d_addrs, (hipStream_t)stream));
    return FB_OK;
}

int fb_flow_count(fb_ctx* c, uint64_t* n_flows, void* stream) {
    if (!c || !n_flows) return set_err(FB_ERR_INVAL, "bad arguments");
    *n_flows = 0;
    if (!c->d_table) return FB_OK;
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    unsigned long long h = 0;
    const int rc = join_updates(c, s);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_n, 0, 8, s));
    HIP_TRY(launch_flow_count(c->d_table, c->table_cap, c->d_n, s));
    HIP_TRY(hipMemcpyAsync(&h, c->d_n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_flows = h;
    return FB_OK;
}

int fb_flow_export_sessions_dev(fb_ctx* c, uint32_t filter, fb_flow_rec* d_out, uint64_t cap, uint64_t* d_n,
                                void* stream) {
    if (!c || !d_n || (cap && !d_out) || filter > FB_FILTER_ALL) return set_err(FB_ERR_INVAL, "bad arguments");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(d_n, 0, 8, s));
    if (!c->d_table) return FB_OK;
    int rc = join_updates(c, s);
    if (!rc && filter != FB_FILTER_ALL) rc = upload_cfg(c, s);  // the LAN configuration as of now
    if (rc) return rc;
    HIP_TRY(launch_flow_export(c->d_table, c->table_cap, d_out, cap, (unsigned long long*)d_n, s, filter, c->d_cfg,
                               c->d_time));
    return FB_OK;
}

int fb_flow_export_times_dev(fb_ctx* c, fb_flow_time* d_out, uint64_t cap, uint64_t* d_n, void* stream) {
    if (!c || !d_n || (cap && !d_out)) return set_err(FB_ERR_INVAL, "bad arguments");
    if (!c->timed) return set_err(FB_ERR_INVAL, "the context was created without FB_CFG_TIMED");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(d_n, 0, 8, s));
    int rc = join_updates(c, s);
    if (rc) return rc;
    HIP_TRY(launch_time_export(c->d_table, c->d_time, c->table_cap, d_out, cap, (unsigned long long*)d_n, s));
    return FB_OK;
}

int fb_flow_export_times(fb_ctx* c, fb_flow_time* out, uint64_t cap, uint64_t* n, void* stream) {
    if (!c || !n || (cap && !out)) return set_err(FB_ERR_INVAL, "bad arguments");
    *n = 0;
    if (!c->timed) return set_err(FB_ERR_INVAL, "the context was created without FB_CFG_TIMED");
    if (cap == 0) return FB_OK;
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    fb_flow_time* d_out = nullptr;
    if (hipMalloc(&d_out, cap * sizeof(fb_flow_time)) != hipSuccess) return set_err(FB_ERR_NOMEM, "export buffer");
    unsigned long long h = 0;
    int rc = fb_flow_export_times_dev(c, d_out, cap, reinterpret_cast<uint64_t*>(c->d_n), stream);
    hipError_t e = rc ? hipSuccess : hipMemcpyAsync(&h, c->d_n, 8, hipMemcpyDeviceToHost, s);
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(s);
    const uint64_t got = std::min<uint64_t>(h, cap);
    if (!rc && e == hipSuccess && got) e = hipMemcpyAsync(out, d_out, got * sizeof(fb_flow_time), hipMemcpyDeviceToHost, s);
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d_out);
    if (rc) return rc;
    if (e != hipSuccess) return set_err(FB_ERR_HIP, "time export: %s", hipGetErrorString(e));
    *n = got;
    return FB_OK;
}

int fb_flow_export_dev(fb_ctx* c, fb_flow_rec* d_out, uint64_t cap, uint64_t* d_n, void* stream) {
    return fb_flow_export_sessions_dev(c, FB_FILTER_ALL, d_out, cap, d_n, stream);
}

// ---- multi-GPU merge (fb_merge.hip) ---------------------------------------------------------------
// The export and the merge share d_mscratch and may be called on different streams: each use waits
// on the event the previous use recorded (mscratch_use / mscratch_done), and a reallocation waits for
// that use on the host before the old buffer is freed.
static int ensure_mscratch(fb_ctx* c, uint64_t bytes, hipStream_t s) {
    if (!c->ev_mscratch) HIP_TRY(hipEventCreateWithFlags(&c->ev_mscratch, hipEventDisableTiming));
    HIP_TRY(hipStreamWaitEvent(s, c->ev_mscratch, 0));  // (an event never recorded is complete)
    if (bytes <= c->mscratch_bytes) return FB_OK;
    HIP_TRY(hipEventSynchronize(c->ev_mscratch));
    HIP_TRY(hipStreamSynchronize(s));
    hipFree(c->d_mscratch);
    c->d_mscratch = nullptr;
    c->mscratch_bytes = 0;
    if (hipMalloc(&c->d_mscratch, bytes) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "merge scratch (%llu bytes)", (unsigned long long)bytes);
    c->mscratch_bytes = bytes;
    return FB_OK;
}

static int export_merge(fb_ctx* c, uint32_t world, uint32_t rank, uint64_t shard_first, const uint64_t* call_map,
                        uint32_t n_calls, fb_flow_mrec* d_out, uint64_t cap, uint64_t* d_counts, void* stream) {
    if (!c || !d_counts || (cap && !d_out)) return set_err(FB_ERR_INVAL, "ctx, d_counts and d_out are required");
    if (world == 0 || world > 64 || rank >= world) return set_err(FB_ERR_INVAL, "1 <= world <= 64, rank < world");
    if (!c->d_table) return set_err(FB_ERR_INVAL, "context was created without a flow table");
    if (call_map) {  // every position the table holds names a call below flow_batch
        if (n_calls < c->flow_batch)
            return set_err(FB_ERR_INVAL, "call map has %u entries, the table holds %u update calls", n_calls,
                           c->flow_batch);
        for (uint32_t k = 0; k < c->flow_batch; ++k) {
            const uint64_t gb = call_map[k] >> 32, first = call_map[k] & 0xFFFFFFFFull;
            if (gb >= 0xFFFFFFFFull || (k && gb <= (call_map[k - 1] >> 32)))
                return set_err(FB_ERR_INVAL, "call map: global batches must increase with the calls (call %u)", k);
            if (first + FB_MAX_BATCH_PACKETS > 0xFFFFFFFFull)
                return set_err(FB_ERR_INVAL, "call map: call %u's shard starts past 2^32 - FB_MAX_BATCH_PACKETS", k);
        }
    }
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    const uint64_t cnt_bytes = merge_export_scratch_bytes(c->table_cap, world);
    int rc = join_updates(c, s);
    if (!rc) rc = ensure_mscratch(c, cnt_bytes + (call_map ? 8ull * std::max<uint32_t>(c->flow_batch, 1u) : 0ull), s);
    if (rc) return rc;
    unsigned long long* d_map = nullptr;
    if (call_map && c->flow_batch) {
        d_map = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->d_mscratch) + cnt_bytes);
        HIP_TRY(hipMemcpyAsync(d_map, call_map, 8ull * c->flow_batch, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(launch_merge_export(c->d_table, c->d_char_call, c->table_cap, world, rank, shard_first,
                                call_map ? d_map : nullptr, d_out, cap, (unsigned long long*)d_counts,
                                c->d_mscratch, s));
    HIP_TRY(hipEventRecord(c->ev_mscratch, s));
    return FB_OK;
}

int fb_flow_export_merge_dev(fb_ctx* c, uint32_t world, uint32_t rank, uint64_t shard_first, fb_flow_mrec* d_out,
                             uint64_t cap, uint64_t* d_counts, void* stream) {
    if (shard_first + FB_MAX_BATCH_PACKETS > 0xFFFFFFFFull)
        return set_err(FB_ERR_INVAL, "shard_first past 2^32 - FB_MAX_BATCH_PACKETS");
    return export_merge(c, world, rank, shard_first, nullptr, 0u, d_out, cap, d_counts, stream);
}

int fb_flow_export_merge_map_dev(fb_ctx* c, uint32_t world, uint32_t rank, const uint64_t* call_map, uint32_t n_calls,
                                 fb_flow_mrec* d_out, uint64_t cap, uint64_t* d_counts, void* stream) {
    if (!call_map && n_calls) return set_err(FB_ERR_INVAL, "call_map is NULL");
    if (!call_map) {  // (a table that took no update call holds no flow)
        static const uint64_t none = 0ull;
        call_map = &none;
    }
    return export_merge(c, world, rank, 0ull, call_map, n_calls, d_out, cap, d_counts, stream);
}

int fb_route_records_dev(fb_ctx* c, const fb_pkt_out* d_recs, const fb_batch_stats* d_stats, uint32_t max_n,
                         uint32_t world, uint64_t shard_first, const uint64_t* d_ts, fb_pkt_out* d_out,
                         uint64_t* d_ts_out, uint64_t* d_counts, void* stream) {
    if (!c || !d_stats || !d_counts || (max_n && (!d_recs || !d_out)))
        return set_err(FB_ERR_INVAL, "ctx, d_stats, d_counts, d_recs and d_out are required");
    if (world == 0 || world > 64) return set_err(FB_ERR_INVAL, "1 <= world <= 64");
    if (max_n > FB_MAX_BATCH_PACKETS) return set_err(FB_ERR_INVAL, "max_n > FB_MAX_BATCH_PACKETS");
    if (shard_first + FB_MAX_BATCH_PACKETS > 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "shard_first too large");
    if ((d_ts == nullptr) != (d_ts_out == nullptr)) return set_err(FB_ERR_INVAL, "d_ts and d_ts_out go together");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    const int rc = ensure_mscratch(c, route_scratch_bytes(max_n, world), s);
    if (rc) return rc;
    HIP_TRY(launch_route(d_recs, d_stats, max_n, world, shard_first, reinterpret_cast<const unsigned long long*>(d_ts),
                         d_out, reinterpret_cast<unsigned long long*>(d_ts_out), (unsigned long long*)d_counts,
                         c->d_mscratch, s));
    HIP_TRY(hipEventRecord(c->ev_mscratch, s));
    return FB_OK;
}

int fb_flow_merge_dev(fb_ctx* c, const fb_flow_mrec* d_in, uint64_t n, fb_flow_rec* d_out, uint64_t* d_n,
                      void* stream) {
    if (!c || !d_n || (n && (!d_in || !d_out))) return set_err(FB_ERR_INVAL, "ctx, d_in, d_out and d_n are required");
    if (n >= 0xFFFFFFFFull) return set_err(FB_ERR_INVAL, "n %llu >= 2^32", (unsigned long long)n);
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    const int rc = ensure_mscratch(c, n ? merge_scratch_bytes(n) : 0, s);
    if (rc) return rc;
    HIP_TRY(launch_merge(d_in, n, d_out, (unsigned long long*)d_n, c->d_mscratch, s));
    HIP_TRY(hipEventRecord(c->ev_mscratch, s));
    return FB_OK;
}

int fb_flow_export_sessions(fb_ctx* c, uint32_t filter, fb_flow_rec* out, uint64_t cap, uint64_t* n, void* stream) {
    if (!c || !n || (cap && !out) || filter > FB_FILTER_ALL) return set_err(FB_ERR_INVAL, "bad arguments");
    *n = 0;
    if (!c->d_table || cap == 0) return FB_OK;
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    uint64_t total = 0;
    int rc = fb_flow_count(c, &total, stream);
    if (!rc && filter != FB_FILTER_ALL) rc = upload_cfg(c, s);
    if (rc) return rc;
    const uint64_t m = std::min(total, cap);
    if (m == 0) return FB_OK;
    fb_flow_rec* d_out = nullptr;
    if (hipMalloc(&d_out, m * sizeof(fb_flow_rec)) != hipSuccess) return set_err(FB_ERR_NOMEM, "export buffer");
    unsigned long long h = 0;
    hipError_t e = hipMemsetAsync(c->d_n, 0, 8, s);
    if (e == hipSuccess) e = launch_flow_export(c->d_table, c->table_cap, d_out, m, c->d_n, s, filter, c->d_cfg, c->d_time);
    if (e == hipSuccess) e = hipMemcpyAsync(&h, c->d_n, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const uint64_t got = std::min<uint64_t>(h, m);
    if (e == hipSuccess && got) e = hipMemcpyAsync(out, d_out, got * sizeof(fb_flow_rec), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d_out);
    if (e != hipSuccess) return set_err(FB_ERR_HIP, "flow export: %s", hipGetErrorString(e));
    *n = got;
    return FB_OK;
}

int fb_flow_export(fb_ctx* c, fb_flow_rec* out, uint64_t cap, uint64_t* n, void* stream) {
    return fb_flow_export_sessions(c, FB_FILTER_ALL, out, cap, n, stream);
}

int fb_flow_table_info_get(fb_ctx* c, fb_flow_table_info* info) {
    if (!c || !info) return set_err(FB_ERR_INVAL, "bad arguments");
    memset(info, 0, sizeof(*info));
    if (!c->d_table) return FB_OK;
    info->capacity = c->table_cap;
    info->partitions = c->flow_parts;
    info->generation = c->generation;
    const volatile FlowMailbox* m = c->h_mbox;
    const uint64_t seq = __atomic_load_n(&m->seq, __ATOMIC_ACQUIRE);
    if (seq && seq > c->clear_seq) {
        info->flows = m->flows;
        info->max_partition = m->max_part;
    }
    return FB_OK;
}

int fb_flow_slot_remap(fb_ctx* c, uint32_t* old_to_new, uint64_t cap, uint64_t* n) {
    if (!c || !n || (cap && !old_to_new)) return set_err(FB_ERR_INVAL, "bad arguments");
    *n = 0;
    if (!c->d_remap || !c->remap_n) return FB_OK;
    DeviceGuard g(c->device);
    const uint64_t m = std::min(cap, c->remap_n);
    if (m) HIP_TRY(hipMemcpy(old_to_new, c->d_remap, m * 4ull, hipMemcpyDeviceToHost));
    *n = m;
    return FB_OK;
}

int fb_flow_clear(fb_ctx* c, void* stream) {
    if (!c) return set_err(FB_ERR_INVAL, "ctx is NULL");
    if (!c->d_table) return FB_OK;
    DeviceGuard g(c->device);
    const int rc = join_updates(c, (hipStream_t)stream);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_table, 0, c->table_cap * sizeof(FlowSlot), (hipStream_t)stream));
    c->flow_batch = 0;
    c->clear_seq = c->upd_seq;
    c->last_recs = nullptr;
    c->last_part = nullptr;
    return FB_OK;
}

// ---- device-memory helpers -------------------------------------------------------------
int fb_dev_alloc(void** p, uint64_t bytes) {
    if (!p) return set_err(FB_ERR_INVAL, "p is NULL");
    *p = nullptr;
    if (hipMalloc(p, bytes ? bytes : 1) != hipSuccess) return set_err(FB_ERR_NOMEM, "hipMalloc(%llu)", (unsigned long long)bytes);
    return FB_OK;
}
int fb_dev_free(void* p) { HIP_TRY(hipFree(p)); return FB_OK; }
int fb_host_alloc_pinned(void** p, uint64_t bytes) {
    if (!p) return set_err(FB_ERR_INVAL, "p is NULL");
    *p = nullptr;
    if (hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return set_err(FB_ERR_NOMEM, "hipHostMalloc(%llu)", (unsigned long long)bytes);
    return FB_OK;
}
int fb_host_free_pinned(void* p) { HIP_TRY(hipHostFree(p)); return FB_OK; }
int fb_memcpy_h2d(void* d, const void* s, uint64_t b, void* st) {
    HIP_TRY(hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, (hipStream_t)st));
    return FB_OK;
}
int fb_memcpy_d2h(void* d, const void* s, uint64_t b, void* st) {
    HIP_TRY(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToHost, (hipStream_t)st));
    return FB_OK;
}
int fb_memset_dev(void* d, int v, uint64_t b, void* st) {
    HIP_TRY(hipMemsetAsync(d, v, b, (hipStream_t)st));
    return FB_OK;
}
int fb_stream_create(void** st) {
    if (!st) return set_err(FB_ERR_INVAL, "NULL");
    HIP_TRY(hipStreamCreateWithFlags((hipStream_t*)st, hipStreamNonBlocking));
    return FB_OK;
}
int fb_stream_destroy(void* st) { HIP_TRY(hipStreamDestroy((hipStream_t)st)); return FB_OK; }
int fb_stream_sync(void* st) { HIP_TRY(hipStreamSynchronize((hipStream_t)st)); return FB_OK; }
int fb_event_create(void** ev) {
    if (!ev) return set_err(FB_ERR_INVAL, "NULL");
    HIP_TRY(hipEventCreate((hipEvent_t*)ev));
    return FB_OK;
}
int fb_event_destroy(void* ev) { HIP_TRY(hipEventDestroy((hipEvent_t)ev)); return FB_OK; }
int fb_event_record(void* ev, void* st) { HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)st)); return FB_OK; }
int fb_event_elapsed_ms(float* ms, void* a, void* b) {
    if (!ms) return set_err(FB_ERR_INVAL, "NULL");
    HIP_TRY(hipEventSynchronize((hipEvent_t)b));
    HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
    return FB_OK;
}
int fb_event_query(void* ev) {
    const hipError_t e = hipEventQuery((hipEvent_t)ev);
    if (e == hipErrorNotReady) return 1;
    HIP_TRY(e);
    return FB_OK;
}
// Busy-wait (no blocking sync, no wake-up latency) until the event completed.
int fb_event_spin(void* ev) {
    for (;;) {
        const hipError_t e = hipEventQuery((hipEvent_t)ev);
        if (e == hipSuccess) return FB_OK;
        if (e != hipErrorNotReady) HIP_TRY(e);
    }
}
int fb_set_device(int d) { HIP_TRY(hipSetDevice(d)); return FB_OK; }

}  // extern "C"
