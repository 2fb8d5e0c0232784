// fb_ring.hip -- host ingest ring.
//
// Replaces the reference's per-packet ingest: the pcap reader thread copies every frame into a
// fresh Vec<u8> and sends it through a bounded mpsc(1000) channel to the processor task, which
// drops the packet when the channel is full (src/capture.rs:1016, 1082-1142; async twin
// 1183-1249), then parses and upserts it one at a time.  Here the reader appends frames into the
// current batch of a ring of page-locked (pinned) batches; a full batch is submitted as one
// pipeline step -- H2D of frames + offsets on a copy stream, then parse + classify + session-table
// upsert (fb_process_seg_dev) on the context's compute stream, then the batch stats (and the DNS side
// records, if any) back -- while the reader fills the next batch.  When every batch is in flight
// the reader waits for the oldest one instead of dropping packets.  The session table stays in
// HBM (read with fb_flow_export), so per frame only its bytes and offset cross PCIe.
//
// Single-threaded like the reference's per-interface processor task: one ring per context, one
// producer thread -- which may split each block's copy over copy_threads helper threads
// (fb_ring_config.copy_threads).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "fb_host.h"

using namespace fbk;

namespace {

struct RingSlot {
    uint8_t* h_frames = nullptr;
    uint32_t* h_offsets = nullptr;
    fb_dns_out* h_dns = nullptr;
    fb_batch_stats* h_stats = nullptr;
    uint8_t* d_frames = nullptr;
    uint32_t* d_offsets = nullptr;
    fb_pkt_out* d_out = nullptr;   // segmented records (ceil(max_packets / 64) * 64 slots)
    uint32_t* d_seg = nullptr;     // segment counts
    fb_dns_out* d_dns = nullptr;   // the batch's DNS side records, compacted
    fb_batch_stats* d_stats = nullptr;
    hipEvent_t ev_h2d = nullptr, ev_done = nullptr;
    uint32_t n = 0;
    uint64_t bytes = 0;
    uint64_t seq0 = 0;   // ring-wide index of the batch's first frame
    bool in_flight = false;
};

// Helper threads of fb_ring_push_block (fb_ring_config.copy_threads - 1 of them): a block's frames
// are split into equal frame ranges, the producer thread taking the first; each thread copies its
// range's bytes into the pinned batch and writes its offsets.  One host thread's memcpy from
// pageable memory moves ~18-20 GB/s (the round-5 copy producer), below PCIe's ~54 GB/s.
class CopyPool {
  public:
    explicit CopyPool(uint32_t helpers) {
        for (uint32_t t = 0; t < helpers; ++t) th_.emplace_back([this, t] { loop(t + 1u); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    uint32_t threads() const { return (uint32_t)th_.size() + 1u; }
    // fn(part, parts) on every thread (part 0 on the caller); returns once all parts are done
    template <class F>
    void run(const F& fn) {
        const uint32_t parts = threads();
        if (parts == 1u) {
            fn(0u, 1u);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = [&fn, parts](uint32_t part) { fn(part, parts); };
            pending_ = parts - 1u;
            ++gen_;
        }
        cv_.notify_all();
        fn(0u, parts);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0u; });
        job_ = nullptr;
    }

  private:
    void loop(uint32_t part) {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(uint32_t)> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
            }
            job(part);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (--pending_ == 0u) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::function<void(uint32_t)> job_;
    uint64_t gen_ = 0;
    uint32_t pending_ = 0;
    bool stop_ = false;
};

}  // namespace

struct fb_ring {
    fb_ctx* ctx = nullptr;
    int device = 0;
    fb_ring_config cfg{};
    std::vector<RingSlot> slots;
    uint32_t cur = 0;          // the batch being filled
    hipStream_t copy = nullptr, compute = nullptr;
    hipStream_t dnsq = nullptr;  // DNS side-record read-back (never queued behind later H2D copies)
    fb_batch_stats total{};
    uint64_t batches = 0;
    uint64_t seq = 0;          // frames accepted so far
    std::vector<fb_ring_dns> dns;  // DNS side records of completed batches, payloads in dns_bytes
    size_t dns_head = 0;
    std::vector<uint8_t> dns_bytes;
    size_t dns_bytes_head = 0;
    CopyPool* pool = nullptr;  // copy_threads > 1
};

namespace {

void free_slot(RingSlot& s) {
    (void)hipHostFree(s.h_frames);
    (void)hipHostFree(s.h_offsets);
    (void)hipHostFree(s.h_dns);
    (void)hipHostFree(s.h_stats);
    (void)hipFree(s.d_frames);
    (void)hipFree(s.d_offsets);
    (void)hipFree(s.d_out);
    (void)hipFree(s.d_seg);
    (void)hipFree(s.d_dns);
    (void)hipFree(s.d_stats);
    if (s.ev_h2d) (void)hipEventDestroy(s.ev_h2d);
    if (s.ev_done) (void)hipEventDestroy(s.ev_done);
    s = RingSlot();
}

bool alloc_slot(RingSlot& s, const fb_ring_config& c) {
    const uint64_t np = c.max_packets;
    const uint64_t nseg = (np + FB_SEG_FRAMES - 1) / FB_SEG_FRAMES;
    return hipHostMalloc((void**)&s.h_frames, std::max<uint64_t>(c.max_bytes, 1), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&s.h_offsets, (np + 1) * 4, hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&s.h_dns, np * sizeof(fb_dns_out), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&s.h_stats, sizeof(fb_batch_stats), hipHostMallocDefault) == hipSuccess &&
           hipMalloc((void**)&s.d_frames, std::max<uint64_t>(c.max_bytes, 1)) == hipSuccess &&
           hipMalloc((void**)&s.d_offsets, (np + 1) * 4) == hipSuccess &&
           hipMalloc((void**)&s.d_out, nseg * FB_SEG_FRAMES * sizeof(fb_pkt_out)) == hipSuccess &&
           hipMalloc((void**)&s.d_seg, nseg * 4) == hipSuccess &&
           hipMalloc((void**)&s.d_dns, np * sizeof(fb_dns_out)) == hipSuccess &&
           hipMalloc((void**)&s.d_stats, sizeof(fb_batch_stats)) == hipSuccess &&
           hipEventCreateWithFlags(&s.ev_h2d, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&s.ev_done, hipEventDisableTiming) == hipSuccess;
}

void add_stats(fb_batch_stats& t, const fb_batch_stats& b) {
    t.total_processed += b.total_processed;
    t.tcp_processed += b.tcp_processed;
    t.udp_processed += b.udp_processed;
    t.ipv4_processed += b.ipv4_processed;
    t.ipv6_processed += b.ipv6_processed;
    t.new_sessions += b.new_sessions;
    t.updated_sessions += b.updated_sessions;
    t.n_session += b.n_session;
    t.n_dns += b.n_dns;
    t.n_drop += b.n_drop;
    t.n_filtered += b.n_filtered;
    t.bad_offsets += b.bad_offsets;
    t.error |= b.error;
}

// Wait for an in-flight batch and retire it: stats into the totals, DNS side records (with
// their payload bytes, still in the slot's pinned frames) into the DNS queue.
int complete(fb_ring* r, RingSlot& s) {
    if (!s.in_flight) return FB_OK;
    HIP_TRY(hipEventSynchronize(s.ev_done));
    s.in_flight = false;
    const fb_batch_stats st = *s.h_stats;
    add_stats(r->total, st);
    r->batches++;
    const uint64_t nd = std::min<uint64_t>(st.n_dns, s.n);
    if (nd) {
        HIP_TRY(hipMemcpyAsync(s.h_dns, s.d_dns, nd * sizeof(fb_dns_out), hipMemcpyDeviceToHost, r->dnsq));
        HIP_TRY(hipStreamSynchronize(r->dnsq));
        for (uint64_t k = 0; k < nd; ++k) {
            const fb_dns_out& d = s.h_dns[k];
            fb_ring_dns x{};
            x.packet_seq = s.seq0 + d.pkt_index;
            x.payload_offset = r->dns_bytes.size();
            x.payload_length = d.payload_length;
            x.protocol = d.protocol;
            x.family = d.family;
            r->dns.push_back(x);
            r->dns_bytes.insert(r->dns_bytes.end(), s.h_frames + d.payload_offset,
                                s.h_frames + d.payload_offset + d.payload_length);
        }
    }
    s.n = 0;
    s.bytes = 0;
    if (st.error) return ctx_report_error(r->ctx, st.error);
    return FB_OK;
}

// Submit the batch being filled (if any) and make the next slot the filling one, retiring it
// first if it is still in flight (the producer waits instead of dropping).
int submit(fb_ring* r) {
    RingSlot& s = r->slots[r->cur];
    int rc = FB_OK;
    if (s.n) {
        s.h_offsets[s.n] = (uint32_t)s.bytes;
        HIP_TRY(hipMemcpyAsync(s.d_frames, s.h_frames, s.bytes, hipMemcpyHostToDevice, r->copy));
        HIP_TRY(hipMemcpyAsync(s.d_offsets, s.h_offsets, (uint64_t)(s.n + 1) * 4, hipMemcpyHostToDevice, r->copy));
        HIP_TRY(hipEventRecord(s.ev_h2d, r->copy));
        HIP_TRY(hipStreamWaitEvent(r->compute, s.ev_h2d, 0));
        // segmented parse (+ session upsert), then only the DNS side records compacted for the
        // read-back: no kernel of the step waits on another workgroup
        rc = (r->cfg.flags & FB_RING_NO_FLOW)
                 ? fb_parse_classify_seg_dev(r->ctx, s.d_frames, s.bytes, s.d_offsets, s.n, s.d_out, s.d_seg, nullptr,
                                             s.d_stats, r->compute)
                 : fb_process_seg_dev(r->ctx, s.d_frames, s.bytes, s.d_offsets, s.n, s.d_out, s.d_seg, nullptr,
                                      s.d_stats, r->compute);
        if (!rc) rc = fb_seg_compact_dev(r->ctx, s.d_out, s.d_seg, s.n, nullptr, s.d_dns, r->compute);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(s.h_stats, s.d_stats, sizeof(fb_batch_stats), hipMemcpyDeviceToHost, r->compute));
        HIP_TRY(hipEventRecord(s.ev_done, r->compute));
        s.in_flight = true;
        r->cur = (r->cur + 1) % (uint32_t)r->slots.size();
    }
    RingSlot& next = r->slots[r->cur];
    if (next.in_flight) rc = complete(r, next);
    if (!next.in_flight && next.n == 0) next.seq0 = r->seq;
    return rc;
}

// Room for one more frame of `caplen` bytes in the filling batch (submitting it when full).
int make_room(fb_ring* r, uint32_t caplen) {
    if (caplen > r->cfg.max_bytes) return set_err(FB_ERR_INVAL, "frame of %u bytes > max_bytes", caplen);
    const RingSlot& s = r->slots[r->cur];
    if (s.n == r->cfg.max_packets || s.bytes + caplen > r->cfg.max_bytes) return submit(r);
    return FB_OK;
}

}  // namespace

extern "C" {

fb_ring* fb_ring_create(fb_ctx* ctx, const fb_ring_config* cfg) {
    if (!ctx || !cfg) { set_err(FB_ERR_INVAL, "ctx and cfg are required"); return nullptr; }
    fb_ring_config c = *cfg;
    if (c.slots == 0) c.slots = 4;
    if (c.slots < 2 || c.slots > 64 || c.max_packets == 0 || c.max_packets > FB_MAX_BATCH_PACKETS ||
        c.max_bytes == 0 || c.max_bytes > 0xFFFFFFFFull) {
        set_err(FB_ERR_INVAL, "ring: 2 <= slots <= 64, 1 <= max_packets <= FB_MAX_BATCH_PACKETS, "
                              "1 <= max_bytes < 4 GiB");
        return nullptr;
    }
    DeviceGuard g(ctx_device(ctx));
    fb_ring* r = new (std::nothrow) fb_ring();
    if (!r) { set_err(FB_ERR_NOMEM, "fb_ring"); return nullptr; }
    r->ctx = ctx;
    r->device = ctx_device(ctx);
    r->cfg = c;
    if (c.copy_threads > 1u) r->pool = new (std::nothrow) CopyPool(std::min<uint32_t>(c.copy_threads, 64u) - 1u);
    r->slots.resize(c.slots);
    bool ok = hipStreamCreateWithFlags(&r->copy, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&r->compute, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&r->dnsq, hipStreamNonBlocking) == hipSuccess;
    ok = ok && (c.copy_threads <= 1u || r->pool);
    for (auto& s : r->slots) ok = ok && alloc_slot(s, c);
    if (!ok) {
        fb_ring_destroy(r);
        set_err(FB_ERR_NOMEM, "ring buffers (%u slots x %llu bytes)", c.slots, (unsigned long long)c.max_bytes);
        return nullptr;
    }
    return r;
}

int fb_ring_destroy(fb_ring* r) {
    if (!r) return set_err(FB_ERR_INVAL, "ring is NULL");
    DeviceGuard g(r->device);
    if (r->compute) (void)hipStreamSynchronize(r->compute);
    if (r->copy) (void)hipStreamSynchronize(r->copy);
    for (auto& s : r->slots) free_slot(s);
    if (r->copy) (void)hipStreamDestroy(r->copy);
    if (r->compute) (void)hipStreamDestroy(r->compute);
    if (r->dnsq) (void)hipStreamDestroy(r->dnsq);
    delete r->pool;
    delete r;
    return FB_OK;
}

uint8_t* fb_ring_reserve(fb_ring* r, uint32_t caplen) {
    if (!r) { set_err(FB_ERR_INVAL, "ring is NULL"); return nullptr; }
    DeviceGuard g(r->device);
    if (make_room(r, caplen)) return nullptr;
    RingSlot& s = r->slots[r->cur];
    uint8_t* p = s.h_frames + s.bytes;
    s.h_offsets[s.n++] = (uint32_t)s.bytes;
    s.bytes += caplen;
    r->seq++;
    return p;
}

uint8_t* fb_ring_reserve_block(fb_ring* r, uint32_t n, uint64_t bytes, uint32_t** offsets, uint32_t* base) {
    if (!r || !offsets || !base || n == 0 || n > r->cfg.max_packets || bytes > r->cfg.max_bytes) {
        set_err(FB_ERR_INVAL, "reserve_block: 1 <= n <= max_packets, bytes <= max_bytes, offsets/base required");
        return nullptr;
    }
    DeviceGuard g(r->device);
    const RingSlot& f = r->slots[r->cur];
    if (f.n + n > r->cfg.max_packets || f.bytes + bytes > r->cfg.max_bytes) {
        if (submit(r)) return nullptr;
    }
    RingSlot& s = r->slots[r->cur];
    uint8_t* p = s.h_frames + s.bytes;
    *offsets = s.h_offsets + s.n;
    *base = (uint32_t)s.bytes;
    s.n += n;
    s.bytes += bytes;
    r->seq += n;
    return p;
}

int fb_ring_push(fb_ring* r, const uint8_t* frame, uint32_t caplen) {
    if (!r || (caplen && !frame)) return set_err(FB_ERR_INVAL, "bad arguments");
    {
        // the per-frame fast path: room in the filling batch -- no device call, so no device guard
        // (hipGetDevice / hipSetDevice cost more than the 64-B copy)
        RingSlot& s = r->slots[r->cur];
        if (s.n < r->cfg.max_packets && s.bytes + caplen <= r->cfg.max_bytes) {
            uint8_t* p = s.h_frames + s.bytes;
            s.h_offsets[s.n++] = (uint32_t)s.bytes;
            s.bytes += caplen;
            r->seq++;
            if (caplen) memcpy(p, frame, caplen);
            return FB_OK;
        }
    }
    uint8_t* p = fb_ring_reserve(r, caplen);
    if (!p) return FB_ERR_INVAL;
    if (caplen) memcpy(p, frame, caplen);
    return FB_OK;
}

int fb_ring_push_block(fb_ring* r, const uint8_t* frames, const uint32_t* offsets, uint32_t n) {
    if (!r || (n && (!frames || !offsets))) return set_err(FB_ERR_INVAL, "bad arguments");
    {
        // validate before any frame is taken (a failed push leaves the ring as it was)
        std::atomic<uint32_t> bad{0xFFFFFFFFu};
        auto check = [&](uint32_t part, uint32_t parts) {
            const uint32_t k0 = (uint32_t)((uint64_t)n * part / parts), k1 = (uint32_t)((uint64_t)n * (part + 1u) / parts);
            for (uint32_t k = k0; k < k1; ++k)
                if (offsets[k + 1] < offsets[k]) {
                    uint32_t cur = bad.load();
                    while (k < cur && !bad.compare_exchange_weak(cur, k)) {}
                    return;
                }
        };
        if (r->pool && n >= (1u << 16)) r->pool->run(check); else check(0u, 1u);
        if (bad.load() != 0xFFFFFFFFu) return set_err(FB_ERR_INVAL, "offsets decrease at %u", bad.load());
    }
    DeviceGuard g(r->device);
    uint32_t i = 0;
    while (i < n) {
        int rc = make_room(r, offsets[i + 1] - offsets[i]);
        if (rc) return rc;
        RingSlot& s = r->slots[r->cur];
        // as many whole frames as fit in this batch, copied in one memcpy
        uint32_t j = i;
        const uint64_t room = r->cfg.max_bytes - s.bytes;
        const uint32_t pk = r->cfg.max_packets - s.n;
        while (j < n && j - i < pk && (uint64_t)offsets[j + 1] - offsets[i] <= room) ++j;
        const uint64_t len = (uint64_t)offsets[j] - offsets[i];
        // frames [i, j): their bytes in one run, their offsets rebased (split over the copy threads
        // by frame ranges for a large run)
        uint8_t* dst = s.h_frames + s.bytes;
        uint32_t* doff = s.h_offsets + s.n;
        const uint64_t rebase = s.bytes;
        const uint32_t i0 = i, cnt = j - i;
        auto copy = [&](uint32_t part, uint32_t parts) {
            const uint32_t a = i0 + (uint32_t)((uint64_t)cnt * part / parts);
            const uint32_t b = i0 + (uint32_t)((uint64_t)cnt * (part + 1u) / parts);
            if (a == b) return;
            memcpy(dst + (offsets[a] - offsets[i0]), frames + offsets[a], (uint64_t)offsets[b] - offsets[a]);
            for (uint32_t k = a; k < b; ++k) doff[k - i0] = (uint32_t)(rebase + offsets[k] - offsets[i0]);
        };
        if (r->pool && len >= (1u << 20)) r->pool->run(copy); else copy(0u, 1u);
        s.n += j - i;
        s.bytes += len;
        r->seq += j - i;
        i = j;
    }
    return FB_OK;
}

int fb_ring_submit(fb_ring* r) {
    if (!r) return set_err(FB_ERR_INVAL, "ring is NULL");
    DeviceGuard g(r->device);
    return submit(r);
}

int fb_ring_sync(fb_ring* r) {
    if (!r) return set_err(FB_ERR_INVAL, "ring is NULL");
    DeviceGuard g(r->device);
    int rc = submit(r);
    const uint32_t m = (uint32_t)r->slots.size();
    for (uint32_t k = 0; k < m; ++k) {  // oldest first
        int e = complete(r, r->slots[(r->cur + k) % m]);
        if (!rc) rc = e;
    }
    return rc;
}

int fb_ring_stats(fb_ring* r, fb_batch_stats* total, uint64_t* batches, uint64_t* frames) {
    if (!r) return set_err(FB_ERR_INVAL, "ring is NULL");
    if (total) *total = r->total;
    if (batches) *batches = r->batches;
    if (frames) *frames = r->seq;
    return FB_OK;
}

int fb_ring_poll_dns(fb_ring* r, fb_ring_dns* out, uint32_t cap, uint8_t* payload, uint64_t payload_cap,
                     uint32_t* n, uint64_t* n_bytes) {
    if (!r || !n || (cap && !out)) return set_err(FB_ERR_INVAL, "bad arguments");
    uint32_t k = 0;
    uint64_t used = 0;
    while (k < cap && r->dns_head < r->dns.size()) {
        const fb_ring_dns& d = r->dns[r->dns_head];
        if (used + d.payload_length > payload_cap) break;
        if (d.payload_length) memcpy(payload + used, r->dns_bytes.data() + d.payload_offset, d.payload_length);
        out[k] = d;
        out[k].payload_offset = used;
        used += d.payload_length;
        r->dns_bytes_head = d.payload_offset + d.payload_length;
        ++r->dns_head;
        ++k;
    }
    if (r->dns_head == r->dns.size()) {  // drained: reuse the queue's storage
        r->dns.clear();
        r->dns_bytes.clear();
        r->dns_head = r->dns_bytes_head = 0;
    }
    *n = k;
    if (n_bytes) *n_bytes = used;
    return FB_OK;
}

}  // extern "C"
