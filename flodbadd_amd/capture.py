"""Host-side mirror of the reference's packet path surface, driving the C ABI.

`FlodbaddGpuCapture` stands where `FlodbaddCapture` (src/capture.rs:70-2030) feeds frames to
`parse_packet_pcap` + `process_parsed_packet` (src/capture.rs:1036-1061): it owns one fb_ctx
(one per capture interface, like the reference's one processor task per interface), exposes
the same knobs (`set_filter`/`get_filter`, capture.rs:185; own IPs, capture.rs:964-970;
`init_local_cache`-style IPv6 LAN prefixes, ip.rs:164-191), and turns batches of frames into
session records, DNS diversions and per-flow counters on the GPU.

There is no CPU path: every method calls libflodbadd_gpu.so, which requires a gfx950 device.
"""
import ctypes as C
import ipaddress

import numpy as np

from . import _native as N
from .sessions import SessionFilter, flows_to_sessions, ip_to_words


def lan_v6_table(prefixes):
    """[(ipv6 address, prefix_len)] -> fb_lan_v6 array (apply_mask_v6, src/ip.rs:44-51)."""
    t = np.zeros(len(prefixes), dtype=N.LAN_V6_DTYPE)
    for i, (ip, pfx) in enumerate(prefixes):
        net = ipaddress.IPv6Network("%s/%d" % (ipaddress.IPv6Address(ip), pfx), strict=False)
        t[i]["net"] = ip_to_words(net.network_address)[0]
        t[i]["prefix"] = pfx
    return t


def own_ip_table(ips):
    t = np.zeros(len(ips), dtype=N.FB_IP_DTYPE)
    for i, ip in enumerate(ips):
        w, fam = ip_to_words(ip)
        t[i]["addr"] = w
        t[i]["family"] = fam
    return t


class BatchResult:
    def __init__(self, records, dns, cls, stats):
        self.records = records  # PKT_OUT_DTYPE, packet order
        self.dns = dns          # DNS_OUT_DTYPE, packet order
        self.cls = cls          # uint8 per frame (fb_class)
        self.stats = stats      # dict of fb_batch_stats


def stats_dict(arr):
    return {k: int(arr[0][k]) for k in N.STATS_FIELDS if not k.startswith("reserved")}


class FlodbaddGpuCapture:
    def __init__(self, device=0, session_filter=SessionFilter.GlobalOnly, flow_capacity=1 << 20,
                 service_bitmap=None, lan_v6=(), own_ips=(), max_batch_packets=1 << 20, track_history=False,
                 grow=True, timed=False):
        """timed: capture-time session state (FB_CFG_TIMED): every batch then comes with its frames'
        capture timestamps (`ts`, ns) and the sessions carry start / last / end times and the
        segment state with the reference's 5-s timeout (src/packets.rs:137-200)."""
        lib = N.gpu_lib()
        self._keep = []
        cfg = N.FbConfig()
        cfg.abi_version = N.FB_ABI_VERSION
        cfg.filter = int(session_filter)
        if service_bitmap is not None:
            bm = np.ascontiguousarray(np.frombuffer(bytes(service_bitmap), dtype=np.uint8))
            if bm.size != 8192:
                raise ValueError("service bitmap must be 8192 bytes (one bit per port), got %d" % bm.size)
            self._keep.append(bm)
            cfg.service_bitmap = bm.ctypes.data
        lt = lan_v6_table(list(lan_v6))
        ot = own_ip_table(list(own_ips))
        self._keep += [lt, ot]
        cfg.lan_v6 = lt.ctypes.data if len(lt) else None
        cfg.n_lan_v6 = len(lt)
        cfg.own_ips = ot.ctypes.data if len(ot) else None
        cfg.n_own_ips = len(ot)
        cfg.flow_capacity = int(flow_capacity)
        cfg.max_batch_packets = int(max_batch_packets)
        cfg.flags = (0 if grow else N.FB_CFG_FIXED_TABLE) | (N.FB_CFG_TIMED if timed else 0)  # (the map is unbounded)
        ctx = lib.fb_create(int(device), C.byref(cfg))
        if not ctx:
            raise N.FbError(N.FB_ERR_NODEV, lib.fb_last_error().decode(errors="replace"))
        self.ctx = C.c_void_p(ctx)
        self.filter = SessionFilter(session_filter)
        self.device = device
        self.flow_capacity = flow_capacity
        self.timed = bool(timed)
        # history strings (src/packets.rs:187-198, 410-426) per table slot, appended batch by batch
        # from fb_flow_history_dev when track_history is set
        self.track_history = bool(track_history) and flow_capacity > 0
        self.histories = {}
        self._generation = 0  # table growths seen (slots move when the table grows)

    # ---- configuration -------------------------------------------------------------------
    def set_filter(self, flt):
        N.check(N.gpu_lib().fb_set_filter(self.ctx, int(flt)))
        self.filter = SessionFilter(flt)

    def get_filter(self):
        return self.filter

    def set_service_bitmap(self, bitmap):
        bm = np.ascontiguousarray(np.frombuffer(bytes(bitmap), dtype=np.uint8))
        if bm.size != 8192:
            raise ValueError("service bitmap must be 8192 bytes (one bit per port), got %d" % bm.size)
        N.check(N.gpu_lib().fb_set_service_bitmap(self.ctx, N.ptr(bm)))

    def set_lan_v6(self, prefixes):
        t = lan_v6_table(list(prefixes))
        N.check(N.gpu_lib().fb_set_lan_v6(self.ctx, N.ptr(t) if len(t) else None, len(t)))

    def set_own_ips(self, ips):
        t = own_ip_table(list(ips))
        N.check(N.gpu_lib().fb_set_own_ips(self.ctx, N.ptr(t) if len(t) else None, len(t)))

    # ---- packet path -----------------------------------------------------------------------
    def _frame_times(self, ts, n):
        """Upload a batch's capture timestamps and hand them to the next update call (timed
        contexts); returns the device buffer (kept alive by the caller until the call is done)."""
        if not self.timed:
            if ts is not None:
                raise ValueError("capture timestamps need a timed capture (timed=True)")
            return None
        if ts is None:
            raise ValueError("a timed capture needs each batch's capture timestamps (ts)")
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        if ts.size < n:
            raise ValueError("%d timestamps for %d frames" % (ts.size, n))
        d = N.DeviceBuffer(max(ts.nbytes, 8))
        if ts.size:
            d.upload(ts)
        N.check(N.gpu_lib().fb_set_frame_times(self.ctx, d.ptr))
        return d

    def parse_classify(self, frames, offsets):
        """Host-memory batch: parse_packet_pcap + per-packet classification for every frame."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = offsets.size - 1
        out = np.zeros(max(n, 1), dtype=N.PKT_OUT_DTYPE)
        dns = np.zeros(max(n, 1), dtype=N.DNS_OUT_DTYPE)
        cls = np.zeros(max(n, 1), dtype=np.uint8)
        st = np.zeros(1, dtype=N.STATS_DTYPE)
        n_out, n_dns = C.c_uint32(0), C.c_uint32(0)
        N.check(N.gpu_lib().fb_parse_classify(self.ctx, N.ptr(frames), frames.nbytes, N.ptr(offsets), n,
                                              N.ptr(out), C.byref(n_out), N.ptr(dns), C.byref(n_dns),
                                              N.ptr(cls), N.ptr(st), None))
        return BatchResult(out[: n_out.value], dns[: n_dns.value], cls[:n], stats_dict(st))

    def process_parsed(self, packets, ts=None):
        """process_parsed_packet (src/packets.rs:202-537) for a batch of SessionPacketData (list)
        or PARSED_DTYPE records: canonical keys + filter on the GPU, then the session-table upsert
        when the capture has a flow table.  Returns a BatchResult (records, cls, stats)."""
        from .sessions import packets_to_parsed
        arr = packets if isinstance(packets, np.ndarray) else packets_to_parsed(list(packets))
        arr = np.ascontiguousarray(arr, dtype=N.PARSED_DTYPE)
        n = arr.size
        out = np.zeros(max(n, 1), dtype=N.PKT_OUT_DTYPE)
        cls = np.zeros(max(n, 1), dtype=np.uint8)
        st = np.zeros(1, dtype=N.STATS_DTYPE)
        n_out = C.c_uint32(0)
        d_ts = self._frame_times(ts, n) if self.flow_capacity else None  # (indexed by pkt_index)
        N.check(N.gpu_lib().fb_process_parsed(self.ctx, N.ptr(arr) if n else None, n, N.ptr(out), C.byref(n_out),
                                              N.ptr(cls), N.ptr(st), None))
        self._pull_history(n)
        return BatchResult(out[: n_out.value], np.zeros(0, dtype=N.DNS_OUT_DTYPE), cls[:n], stats_dict(st))

    def process_frames(self, frames, offsets, ts=None):
        """parse + classify + flow-table upsert (the whole process_parsed_packet per frame); ts: the
        frames' capture timestamps (ns) on a timed capture."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = offsets.size - 1
        lib = N.gpu_lib()
        d_fr = N.DeviceBuffer(max(frames.nbytes, 1)).upload(frames) if frames.nbytes else N.DeviceBuffer(1)
        d_off = N.DeviceBuffer(offsets.nbytes).upload(offsets)
        d_out = N.DeviceBuffer(max(n, 1) * N.PKT_OUT_DTYPE.itemsize)
        d_dns = N.DeviceBuffer(max(n, 1) * N.DNS_OUT_DTYPE.itemsize)
        d_cls = N.DeviceBuffer(max(n, 1))
        d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        d_ts = self._frame_times(ts, n)  # noqa: F841 (alive until the call's results are read)
        N.check(lib.fb_process_dev(self.ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr,
                                   d_cls.ptr, d_st.ptr, None))
        st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        sd = stats_dict(st)
        out = d_out.download(np.zeros(max(sd["n_session"], 1), dtype=N.PKT_OUT_DTYPE),
                             sd["n_session"] * N.PKT_OUT_DTYPE.itemsize)[: sd["n_session"]]
        dns = d_dns.download(np.zeros(max(sd["n_dns"], 1), dtype=N.DNS_OUT_DTYPE),
                             sd["n_dns"] * N.DNS_OUT_DTYPE.itemsize)[: sd["n_dns"]]
        cls = d_cls.download(np.zeros(max(n, 1), dtype=np.uint8), n)[:n]
        if sd["error"]:
            e = sd["error"]
            code = N.FB_ERR_TABLE_FULL if e & 4 else N.FB_ERR_INTERNAL
            raise N.FbError(code, "device error word %d" % e)
        self._pull_history(n)
        return BatchResult(out, dns, cls, sd)

    def process_frames_seg(self, frames, offsets, flow=True, ts=None):
        """The segmented streaming path (fb_process_seg_dev / fb_parse_classify_seg_dev): same
        classification and session-table update, records left in per-wavefront segments on the
        device; returned here densified (packet order) for comparison with process_frames."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = offsets.size - 1
        nseg = max((n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES, 1)
        lib = N.gpu_lib()
        d_fr = N.DeviceBuffer(max(frames.nbytes, 1)).upload(frames) if frames.nbytes else N.DeviceBuffer(1)
        d_off = N.DeviceBuffer(offsets.nbytes).upload(offsets)
        d_out = N.DeviceBuffer(nseg * N.SEG_BYTES)
        d_seg = N.DeviceBuffer(nseg * 4)
        d_cls = N.DeviceBuffer(max(n, 1))
        d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        d_ts = self._frame_times(ts, n) if flow else None  # noqa: F841
        fn = lib.fb_process_seg_dev if flow else lib.fb_parse_classify_seg_dev
        N.check(fn(self.ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, d_seg.ptr, d_cls.ptr, d_st.ptr, None))
        sd = stats_dict(d_st.download(np.zeros(1, dtype=N.STATS_DTYPE)))
        if sd["error"]:
            e = sd["error"]
            raise N.FbError(N.FB_ERR_TABLE_FULL if e & 4 else N.FB_ERR_INTERNAL, "device error word %d" % e)
        if flow:
            self._pull_history(((n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES) * N.FB_SEG_FRAMES)
        seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))
        raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
        out, dns = N.seg_unpack(raw, seg[: (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES])
        cls = d_cls.download(np.zeros(max(n, 1), dtype=np.uint8), n)[:n]
        return BatchResult(out, dns, cls, sd)

    # ---- session table -----------------------------------------------------------------------
    def flow_history(self, n_slots):
        """fb_flow_history_dev: the last update's history characters grouped per flow, packet order
        inside each flow -> {table slot: str}.  n_slots = that update's record slots (its batch's
        n frames, dense; ceil(n/64)*64, segmented)."""
        m = max(int(n_slots), 1)
        d_h, d_s, d_n = N.DeviceBuffer(m), N.DeviceBuffer(4 * m), N.DeviceBuffer(4)
        N.check(N.gpu_lib().fb_flow_history_dev(self.ctx, d_h.ptr, d_s.ptr, d_n.ptr, None))
        k = int(d_n.download(np.zeros(1, dtype=np.uint32))[0])
        if k == 0:
            return {}
        chars = d_h.download(np.zeros(k, dtype=np.uint8), k)
        slots = d_s.download(np.zeros(k, dtype=np.uint32), 4 * k)
        cut = np.flatnonzero(np.diff(slots)) + 1
        starts, ends = np.r_[0, cut], np.r_[cut, k]
        return {int(slots[a]): chars[a:b].tobytes().decode("ascii") for a, b in zip(starts, ends)}

    def table_info(self):
        """fb_flow_table_info_get: capacity, partitions, growths, flows / fullest partition as the
        last completed update reported."""
        t = N.FlowTableInfo()
        N.check(N.gpu_lib().fb_flow_table_info_get(self.ctx, C.byref(t)))
        return dict(capacity=t.capacity, partitions=t.partitions, generation=t.generation, flows=t.flows,
                    max_partition=t.max_partition)

    def _follow_growth(self):
        """The table grew since the histories were last keyed: move them to the new slots
        (fb_flow_slot_remap; only the last growth's map is kept, and this runs after every batch)."""
        gen = self.table_info()["generation"]
        if gen == self._generation:
            return
        if gen != self._generation + 1:  # fb_flow_slot_remap keeps only the last growth's map
            raise N.FbError(N.FB_ERR_INTERNAL, "the table grew %d times since the histories were keyed"
                            % (gen - self._generation))
        self._generation = gen
        if not self.histories:
            return
        old_cap = max(self.histories) + 1
        m = np.zeros(max(old_cap, 1), dtype=np.uint32)
        n = C.c_uint64(0)
        N.check(N.gpu_lib().fb_flow_slot_remap(self.ctx, N.ptr(m), old_cap, C.byref(n)))
        self.histories = {int(m[k]): v for k, v in self.histories.items()}

    def _pull_history(self, n_slots):
        if not self.track_history:
            return
        self._follow_growth()
        for slot, run in self.flow_history(n_slots).items():
            self.histories[slot] = self.histories.get(slot, "") + run

    def flow_count(self):
        n = C.c_uint64(0)
        N.check(N.gpu_lib().fb_flow_count(self.ctx, C.byref(n), None))
        return n.value

    def export_flows(self, session_filter=SessionFilter.All):
        """fb_flow_export_sessions: every flow (All), or those passing the filter evaluated now."""
        cnt = self.flow_count()
        out = np.zeros(max(cnt, 1), dtype=N.FLOW_REC_DTYPE)
        n = C.c_uint64(0)
        N.check(N.gpu_lib().fb_flow_export_sessions(self.ctx, int(session_filter), N.ptr(out), cnt, C.byref(n), None))
        return out[: n.value]

    def export_times(self):
        """fb_flow_export_times: every flow's FLOW_TIME_DTYPE record (timed captures), with its slot."""
        cnt = self.flow_count()
        out = np.zeros(max(cnt, 1), dtype=N.FLOW_TIME_DTYPE)
        n = C.c_uint64(0)
        N.check(N.gpu_lib().fb_flow_export_times(self.ctx, N.ptr(out), cnt, C.byref(n), None))
        return out[: n.value]

    def get_sessions(self):
        """get_sessions (src/capture.rs:1578-1612): the sessions that pass the CURRENT filter,
        is_local_session! evaluated at query time on the GPU (capture.rs:1603-1608), sorted by the
        derived Ord of Session (integer counters + derived f64s)."""
        return flows_to_sessions(self.export_flows(self.filter), self.histories if self.track_history else None,
                                 times=self.export_times() if self.timed else None)

    # ---- new-session enrichment (src/packets.rs:429-485) -------------------------------------
    def set_asn_tables(self, v4, v6):
        """ASN_RANGE_DTYPE tables (flodbadd_amd.enrich.asn_tables_from_tsv) -> fb_set_asn_tables."""
        v4 = np.ascontiguousarray(v4, dtype=N.ASN_RANGE_DTYPE)
        v6 = np.ascontiguousarray(v6, dtype=N.ASN_RANGE_DTYPE)
        N.check(N.gpu_lib().fb_set_asn_tables(self.ctx, N.ptr(v4) if len(v4) else None, len(v4),
                                              N.ptr(v6) if len(v6) else None, len(v6)))

    def set_blacklists(self, cidrs):
        """CIDR_DTYPE ranges (flodbadd_amd.enrich.blacklists_from_json) -> fb_set_blacklists."""
        cidrs = np.ascontiguousarray(cidrs, dtype=N.CIDR_DTYPE)
        N.check(N.gpu_lib().fb_set_blacklists(self.ctx, N.ptr(cidrs) if len(cidrs) else None, len(cidrs)))

    def ip_lookup(self, ips):
        """get_asn + is_ip_blacklisted for addresses (strings / ipaddress objects) ->
        (int32 ASN records, -1 = None; uint64 list masks)."""
        t = own_ip_table(list(ips))
        n = len(t)
        d_ip = N.DeviceBuffer(max(t.nbytes, 1))
        if n:
            d_ip.upload(t)
        d_a, d_l = N.DeviceBuffer(max(4 * n, 4)), N.DeviceBuffer(max(8 * n, 8))
        N.check(N.gpu_lib().fb_ip_lookup_dev(self.ctx, d_ip.ptr, n, d_a.ptr, d_l.ptr, None))
        return d_a.download(np.zeros(max(n, 1), dtype=np.int32))[:n], d_l.download(np.zeros(max(n, 1), dtype=np.uint64))[:n]

    def enrich(self, new_only=False):
        """fb_flow_enrich_dev -> FLOW_ENRICH_DTYPE records (slot-keyed; join with export_flows)."""
        cap = max(self.flow_count(), 1)
        d_out, d_n = N.DeviceBuffer(cap * N.FLOW_ENRICH_DTYPE.itemsize), N.DeviceBuffer(8)
        N.check(N.gpu_lib().fb_flow_enrich_dev(self.ctx, 1 if new_only else 0, d_out.ptr, cap, d_n.ptr, None))
        m = min(int(d_n.download(np.zeros(1, dtype=np.uint64))[0]), cap)
        return d_out.download(np.zeros(cap, dtype=N.FLOW_ENRICH_DTYPE))[:m]

    def clear_all_sessions(self):
        """src/capture.rs:396 (`stop()` clears the table, capture.rs:383)."""
        N.check(N.gpu_lib().fb_flow_clear(self.ctx, None))
        N.check(N.gpu_lib().fb_stream_sync(None))
        self.histories = {}

    def close(self):
        if getattr(self, "ctx", None):
            N.gpu_lib().fb_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class IngestRing:
    """fb_ring_* (include/flodbadd_gpu.h): the capture reader's batch ring in front of a
    FlodbaddGpuCapture's context -- replaces the reader -> Vec<u8> -> mpsc(1000) -> processor
    path (src/capture.rs:1016, 1082-1142).  Frames are appended into pinned batches, each full
    batch is copied in, parsed, classified and upserted into the context's session table on the
    GPU while the next one fills; the producer waits (never drops) when every batch is in flight."""

    def __init__(self, capture, slots=4, max_packets=1 << 20, max_bytes=64 << 20, flow=True):
        self.lib = N.gpu_lib()
        cfg = N.FbRingConfig(slots, max_packets, max_bytes, 0 if flow else N.FB_RING_NO_FLOW, 0)
        r = self.lib.fb_ring_create(capture.ctx, C.byref(cfg))
        if not r:
            raise N.FbError(N.FB_ERR_INVAL, self.lib.fb_last_error().decode(errors="replace"))
        self.r = C.c_void_p(r)
        self.capture = capture  # the context must outlive the ring

    def push(self, frame):
        f = np.frombuffer(bytes(frame), dtype=np.uint8)
        N.check(self.lib.fb_ring_push(self.r, N.ptr(f) if f.size else None, f.size))

    def push_block(self, frames, offsets):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        N.check(self.lib.fb_ring_push_block(self.r, N.ptr(frames), N.ptr(offsets), offsets.size - 1))

    def sync(self):
        N.check(self.lib.fb_ring_sync(self.r))

    def stats(self):
        """(PACKET_STATS totals over the completed batches, batches completed, frames pushed)."""
        tot = np.zeros(1, dtype=N.STATS_DTYPE)
        nb, nf = C.c_uint64(), C.c_uint64()
        N.check(self.lib.fb_ring_stats(self.r, N.ptr(tot), C.byref(nb), C.byref(nf)))
        return stats_dict(tot), nb.value, nf.value

    def poll_dns(self, max_records=1 << 16, max_bytes=1 << 24):
        """DNS side records of completed batches: [(packet_seq, protocol, family, payload bytes)]
        -- what the reference hands to process_dns_packet (src/capture.rs:1051-1057)."""
        out = np.zeros(max_records, dtype=N.RING_DNS_DTYPE)
        buf = np.zeros(max_bytes, dtype=np.uint8)
        n, nb = C.c_uint32(), C.c_uint64()
        N.check(self.lib.fb_ring_poll_dns(self.r, N.ptr(out), max_records, N.ptr(buf), max_bytes, C.byref(n),
                                          C.byref(nb)))
        return [(int(d["packet_seq"]), int(d["protocol"]), int(d["family"]),
                 buf[int(d["payload_offset"]): int(d["payload_offset"]) + int(d["payload_length"])].tobytes())
                for d in out[: n.value]]

    def close(self):
        if getattr(self, "r", None):
            self.lib.fb_ring_destroy(self.r)
            self.r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
