"""ctypes binding of include/flodbadd_gpu.h (libflodbadd_gpu.so) + numpy record dtypes.

The GPU library is the product path: there is no CPU fallback.  `gpu_lib()` raises
NativeLibraryMissing if the in-tree .so is absent, and fb_create fails loudly without a gfx950.
"""
import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
GPU_LIB_PATH = os.environ.get("FLODBADD_GPU_LIB") or os.path.join(PKG, "libflodbadd_gpu.so")  # override: tools/
SYNTH_LIB_PATH = os.path.join(PKG, "libfb_synth.so")

FB_ABI_VERSION = 4
FB_MAX_BATCH_PACKETS = (1 << 27) - 1
FB_MAX_LAN_V6 = 64
FB_MAX_OWN_IPS = 64

# fb_err
FB_OK, FB_ERR_INVAL, FB_ERR_NOMEM, FB_ERR_HIP, FB_ERR_NODEV, FB_ERR_TABLE_FULL, FB_ERR_INTERNAL = 0, -1, -2, -3, -4, -5, -6
# fb_filter (SessionFilter discriminants, src/sessions.rs:173-178)
FB_FILTER_LOCAL_ONLY, FB_FILTER_GLOBAL_ONLY, FB_FILTER_ALL = 0, 1, 2
# fb_class
FB_CLASS_SESSION, FB_CLASS_DNS, FB_CLASS_DROP, FB_CLASS_FILTERED = 0, 1, 2, 3
# fb_meta_bits
META_HAS_FLAGS, META_SWAP, META_ORIGINATOR = 1, 2, 4
META_LOCAL_SRC, META_LOCAL_DST, META_SELF_SRC, META_SELF_DST, META_DST_SERVICE = 8, 16, 32, 64, 128

KEY_FIELDS = [("src_ip", "<u4", (4,)), ("dst_ip", "<u4", (4,)), ("src_port", "<u2"), ("dst_port", "<u2"),
              ("protocol", "u1"), ("family", "u1"), ("padding", "<u2")]
PKT_OUT_DTYPE = np.dtype(KEY_FIELDS + [
    ("packet_length", "<u4"), ("ip_packet_length", "<u4"), ("tcp_flags", "u1"), ("meta", "u1"),
    ("hist_char", "u1"), ("reserved", "u1"), ("pkt_index", "<u4")])
PARSED_DTYPE = np.dtype(KEY_FIELDS + [
    ("packet_length", "<u4"), ("ip_packet_length", "<u4"), ("tcp_flags", "u1"), ("has_flags", "u1"),
    ("reserved", "<u2"), ("pkt_index", "<u4")])
DNS_OUT_DTYPE = np.dtype([("pkt_index", "<u4"), ("payload_offset", "<u4"), ("payload_length", "<u4"),
                          ("protocol", "u1"), ("family", "u1"), ("reserved", "<u2")])
STATS_FIELDS = ["total_processed", "tcp_processed", "udp_processed", "ipv4_processed", "ipv6_processed",
                "new_sessions", "updated_sessions", "n_session", "n_dns", "n_drop", "n_filtered",
                "bad_offsets", "error", "reserved0", "reserved1", "reserved2"]
STATS_DTYPE = np.dtype([(f, "<u8") for f in STATS_FIELDS])
FLOW_REC_DTYPE = np.dtype(KEY_FIELDS + [
    ("outbound_bytes", "<u8"), ("inbound_bytes", "<u8"), ("orig_pkts", "<u8"), ("resp_pkts", "<u8"),
    ("orig_ip_bytes", "<u8"), ("resp_ip_bytes", "<u8"),
    ("first_seen", "<u8"), ("last_seen", "<u8"), ("end_seen", "<u8"), ("hist_len", "<u4"),
    ("hist_mask", "<u2"), ("conn_state", "u1"), ("end_mask", "u1"), ("slot", "<u4"), ("session_flags", "<u4"),
    ("segment_count", "<u4"), ("in_segment", "u1"), ("reserved", "u1", (3,))])
# fb_flow_mrec: a flow record exported for the multi-GPU merge (positions global, slot = the rank) and
# the update call of the flow's first S, s, H, h (FB_CALL_NONE: none)
FLOW_MREC_DTYPE = np.dtype([("rec", FLOW_REC_DTYPE), ("char_call", "<u4", (4,))])
FB_CALL_NONE = 0xFFFFFFFF
# fb_flow_time: a flow's capture-time state on a timed context (FB_CFG_TIMED)
FLOW_TIME_DTYPE = np.dtype([
    ("start_time_ns", "<u8"), ("last_activity_ns", "<u8"), ("end_time_ns", "<u8"),
    ("current_segment_start_ns", "<u8"), ("last_segment_end_ns", "<u8"),
    ("total_segment_interarrival_ms", "<i8"), ("segment_interarrival_div", "<u4"), ("segment_count", "<u4"),
    ("in_segment", "u1"), ("reserved", "u1", (3,)), ("slot", "<u4")])
assert FLOW_TIME_DTYPE.itemsize == 64
FB_SEGMENT_TIMEOUT_MS = 5000
FB_CFG_TIMED = 2
FB_QUEUE_SHARED = 1
# fb_session_flags (fb_flow_rec.session_flags: SessionInfo.is_local_src/dst, is_self_src/dst and
# dst_service is Some, at insert)
SESSION_LOCAL_SRC, SESSION_LOCAL_DST, SESSION_SELF_SRC, SESSION_SELF_DST, SESSION_DST_SERVICE = 1, 2, 4, 8, 16
# fb_flow_rec positions: (update call << 32) | pkt_index; FB_SEEN_NONE = None
FB_SEEN_NONE = (1 << 64) - 1
FB_HIST_CHARS = "SsHhFfRr><Aa-"
# fb_conn_state -> determine_conn_state string (src/packets.rs:539-559); 0 = None
CONN_STATES = {0: None, 1: "SF", 2: "S0", 3: "REJ", 4: "S1", 5: "-"}
ASN_RANGE_DTYPE = np.dtype([("start", "<u4", (4,)), ("end", "<u4", (4,)), ("as_number", "<u4"), ("record", "<u4"),
                            ("reserved", "<u4", (2,))])
CIDR_DTYPE = np.dtype([("addr", "<u4", (4,)), ("family", "<u4"), ("prefix", "<u4"), ("list", "<u4"),
                       ("reserved", "<u4")])
FLOW_ENRICH_DTYPE = np.dtype([("slot", "<u4"), ("flags", "<u4"), ("src_asn", "<i4"), ("dst_asn", "<i4"),
                              ("src_blacklists", "<u8"), ("dst_blacklists", "<u8")])
FB_MAX_BLACKLISTS = 64
# fb_dns_msg + constants (include/flodbadd_gpu.h, DNS divert parse)
DNS_MSG_DTYPE = np.dtype([("pkt_index", "<u4"), ("id", "<u2"), ("status", "u1"), ("flags", "u1"),
                          ("questions", "<u2"), ("answers", "<u2"), ("name_len", "<u2"), ("n_addrs", "u1"),
                          ("reserved", "u1")])
FB_DNS_MAX_NAME, FB_DNS_MAX_ADDRS = 256, 8
DNS_QUERY, DNS_HAS_QUESTION, DNS_REVERSE, DNS_NAME_TRUNCATED, DNS_ADDRS_TRUNCATED = 1, 2, 4, 8, 16
DNS_STATUS = ["ok", "header_too_short", "unexpected_eof", "bad_pointer", "unknown_label_format", "label_not_ascii",
              "invalid_query_type", "invalid_query_class", "invalid_type", "invalid_class", "wrong_rdata_length",
              "additional_opt"]
ENRICH_LOCAL_SRC, ENRICH_LOCAL_DST, ENRICH_SELF_SRC, ENRICH_SELF_DST = 1, 2, 4, 8
LAN_V6_DTYPE = np.dtype([("net", "<u4", (4,)), ("prefix", "<u4"), ("reserved", "<u4", (3,))])
FB_IP_DTYPE = np.dtype([("addr", "<u4", (4,)), ("family", "<u4"), ("reserved", "<u4", (3,))])

FB_SEG_FRAMES = 64
SEG_BYTES = FB_SEG_FRAMES * 56
FB_MAX_SEG_BATCHES = 32
FB_QUEUE_MAX_DEPTH = 32
# fb_seg_batch: one batch of fb_parse_classify_seg_batches_dev (device pointers as integers)
SEG_BATCH_DTYPE = np.dtype([("d_frames", "<u8"), ("frames_bytes", "<u8"), ("d_offsets", "<u8"), ("n", "<u4"),
                            ("reserved", "<u4"), ("d_out", "<u8"), ("d_seg", "<u8"), ("d_class", "<u8"),
                            ("d_stats", "<u8")])
assert SEG_BATCH_DTYPE.itemsize == 64


def seg_unpack(out_bytes, seg):
    """Densify a segmented batch (fb_parse_classify_seg_dev layout, include/flodbadd_gpu.h):
    returns (SESSION records, DNS records) in packet order, as the dense call would."""
    out_bytes = np.frombuffer(memoryview(out_bytes), dtype=np.uint8)
    seg = np.asarray(seg, dtype=np.uint32)
    recs, dns = [], []
    for s, w in enumerate(seg.tolist()):
        cs, cd = w & 0xFFFF, w >> 16
        base = s * SEG_BYTES
        if cs:
            recs.append(out_bytes[base: base + cs * 56].view(PKT_OUT_DTYPE))
        if cd:
            tail = out_bytes[base + SEG_BYTES - 16 * cd: base + SEG_BYTES].view(DNS_OUT_DTYPE)
            dns.append(tail[::-1])
    r = np.concatenate(recs) if recs else np.zeros(0, dtype=PKT_OUT_DTYPE)
    d = np.concatenate(dns) if dns else np.zeros(0, dtype=DNS_OUT_DTYPE)
    return r, d


assert PKT_OUT_DTYPE.itemsize == 56 and DNS_OUT_DTYPE.itemsize == 16 and PARSED_DTYPE.itemsize == 56
assert STATS_DTYPE.itemsize == 128 and FLOW_REC_DTYPE.itemsize == 136 and FLOW_MREC_DTYPE.itemsize == 152
assert LAN_V6_DTYPE.itemsize == 32 and FB_IP_DTYPE.itemsize == 32
assert ASN_RANGE_DTYPE.itemsize == 48 and CIDR_DTYPE.itemsize == 32 and FLOW_ENRICH_DTYPE.itemsize == 32
assert DNS_MSG_DTYPE.itemsize == 16


class FbConfig(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("filter", C.c_uint32), ("service_bitmap", C.c_void_p),
                ("lan_v6", C.c_void_p), ("n_lan_v6", C.c_uint32), ("n_own_ips", C.c_uint32),
                ("own_ips", C.c_void_p), ("flow_capacity", C.c_uint64), ("max_batch_packets", C.c_uint32),
                ("flags", C.c_uint32), ("max_batch_bytes", C.c_uint64)]


FB_CFG_FIXED_TABLE = 1
FB_MAX_FLOW_CAPACITY = 1 << 25


class FlowTableInfo(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("partitions", C.c_uint64), ("generation", C.c_uint64),
                ("flows", C.c_uint64), ("max_partition", C.c_uint64), ("reserved", C.c_uint64 * 3)]


class FbRingConfig(C.Structure):
    _fields_ = [("slots", C.c_uint32), ("max_packets", C.c_uint32), ("max_bytes", C.c_uint64),
                ("flags", C.c_uint32), ("copy_threads", C.c_uint32)]


FB_RING_NO_FLOW = 1
RING_DNS_DTYPE = np.dtype([("packet_seq", "<u8"), ("payload_offset", "<u8"), ("payload_length", "<u4"),
                           ("protocol", "u1"), ("family", "u1"), ("reserved", "<u2")])
assert RING_DNS_DTYPE.itemsize == 24


class NativeLibraryMissing(RuntimeError):
    pass


class FbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("fb error %d: %s" % (code, msg))
        self.code = code


# Every symbol include/flodbadd_gpu.h declares: (name, restype, argtypes).
_P, _U32, _U64, _I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
_PU32, _PU64 = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
FB_DEBUG_DENSE_STEAL_POLLS, FB_DEBUG_DENSE_OFFSET_SKEW = 1, 2

GPU_SYMBOLS = [
    ("fb_abi_version", _U32, []),
    ("fb_last_error", C.c_char_p, []),
    ("fb_create", _P, [_I, C.POINTER(FbConfig)]),
    ("fb_destroy", _I, [_P]),
    ("fb_set_filter", _I, [_P, _U32]),
    ("fb_set_service_bitmap", _I, [_P, _P]),
    ("fb_set_lan_v6", _I, [_P, _P, _U32]),
    ("fb_set_own_ips", _I, [_P, _P, _U32]),
    ("fb_set_stage_event", _I, [_P, _P]),
    ("fb_set_session_records", _I, [_P, C.c_int]),
    ("fb_parse_classify_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_parse_classify", _I, [_P, _P, _U64, _P, _U32, _P, _PU32, _P, _PU32, _P, _P, _P]),
    ("fb_process_parsed_dev", _I, [_P, _P, _U32, _P, _P, _P, _P]),
    ("fb_process_parsed", _I, [_P, _P, _U32, _P, _PU32, _P, _P, _P]),
    ("fb_flow_update_dev", _I, [_P, _P, _P, _P]),
    ("fb_process_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_parse_classify_seg_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_process_parsed_seg_dev", _I, [_P, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_seg_compact_dev", _I, [_P, _P, _P, _U32, _P, _P, _P]),
    ("fb_parse_classify_seg_batches_dev", _I, [_P, _P, _U32, _P]),
    ("fb_flow_update_seg_dev", _I, [_P, _P, _P, _U32, _P, _P]),
    ("fb_process_seg_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_process_seg_async_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_flow_join", _I, [_P, _P]),
    ("fb_flow_history_dev", _I, [_P, _P, _P, _P, _P]),
    ("fb_set_asn_tables", _I, [_P, _P, _U32, _P, _U32]),
    ("fb_set_blacklists", _I, [_P, _P, _U32]),
    ("fb_ip_lookup_dev", _I, [_P, _P, _U32, _P, _P, _P]),
    ("fb_flow_enrich_dev", _I, [_P, _U32, _P, _U64, _P, _P]),
    ("fb_dns_parse_dev", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P, _P, _P]),
    ("fb_flow_count", _I, [_P, _PU64, _P]),
    ("fb_flow_export", _I, [_P, _P, _U64, _PU64, _P]),
    ("fb_flow_export_dev", _I, [_P, _P, _U64, _P, _P]),
    ("fb_flow_export_sessions", _I, [_P, _U32, _P, _U64, _PU64, _P]),
    ("fb_flow_export_sessions_dev", _I, [_P, _U32, _P, _U64, _P, _P]),
    ("fb_flow_clear", _I, [_P, _P]),
    ("fb_flow_table_info_get", _I, [_P, C.POINTER(FlowTableInfo)]),
    ("fb_flow_slot_remap", _I, [_P, _P, _U64, _PU64]),
    ("fb_flow_hash", _U64, [_P]),
    ("fb_flow_export_merge_dev", _I, [_P, _U32, _U32, _U64, _P, _U64, _P, _P]),
    ("fb_flow_export_merge_map_dev", _I, [_P, _U32, _U32, _P, _U32, _P, _U64, _P, _P]),
    ("fb_flow_merge_dev", _I, [_P, _P, _U64, _P, _P, _P]),
    ("fb_flow_update_records_dev", _I, [_P, _P, _U32, _P, _P]),
    ("fb_route_records_dev", _I, [_P, _P, _P, _U32, _U32, _U64, _P, _P, _P, _P, _P]),
    ("fb_flow_owner", _U32, [_P, _U32]),
    ("fb_ring_create", _P, [_P, C.POINTER(FbRingConfig)]),
    ("fb_ring_destroy", _I, [_P]),
    ("fb_ring_push", _I, [_P, _P, _U32]),
    ("fb_ring_push_block", _I, [_P, _P, _P, _U32]),
    ("fb_ring_reserve", _P, [_P, _U32]),
    ("fb_ring_reserve_block", _P, [_P, _U32, _U64, C.POINTER(C.c_void_p), _PU32]),
    ("fb_ring_submit", _I, [_P]),
    ("fb_ring_sync", _I, [_P]),
    ("fb_ring_stats", _I, [_P, _P, _PU64, _PU64]),
    ("fb_ring_poll_dns", _I, [_P, _P, _U32, _P, _U64, _PU32, _PU64]),
    ("fb_dev_alloc", _I, [C.POINTER(C.c_void_p), _U64]),
    ("fb_dev_free", _I, [_P]),
    ("fb_host_alloc_pinned", _I, [C.POINTER(C.c_void_p), _U64]),
    ("fb_host_free_pinned", _I, [_P]),
    ("fb_memcpy_h2d", _I, [_P, _P, _U64, _P]),
    ("fb_memcpy_d2h", _I, [_P, _P, _U64, _P]),
    ("fb_memset_dev", _I, [_P, _I, _U64, _P]),
    ("fb_stream_create", _I, [C.POINTER(C.c_void_p)]),
    ("fb_stream_destroy", _I, [_P]),
    ("fb_stream_sync", _I, [_P]),
    ("fb_event_create", _I, [C.POINTER(C.c_void_p)]),
    ("fb_event_destroy", _I, [_P]),
    ("fb_event_record", _I, [_P, _P]),
    ("fb_event_elapsed_ms", _I, [C.POINTER(C.c_float), _P, _P]),
    ("fb_event_query", _I, [_P]),
    ("fb_event_spin", _I, [_P]),
    ("fb_device_count", _I, [C.POINTER(C.c_int)]),
    ("fb_set_device", _I, [_I]),
    ("fb_ctx_device", _I, [_P, C.POINTER(C.c_int)]),
    ("fb_seg_queue_create", _P, [_P, _U32, _U32]),
    ("fb_seg_queue_create_ex", _P, [_P, _U32, _U32, _U32]),
    ("fb_seg_queue_submit", _I, [_P, _P, _PU64]),
    ("fb_seg_queue_query", _I, [_P, _U64]),
    ("fb_seg_queue_wait", _I, [_P, _U64]),
    ("fb_seg_queue_destroy", _I, [_P]),
    ("fb_seg_queue_set_limit", _I, [_P, _U64]),
    ("fb_debug_set", _I, [_P, _U32, _U64]),
    ("fb_set_frame_times", _I, [_P, _P]),
    ("fb_flow_export_times_dev", _I, [_P, _P, _U64, _P, _P]),
    ("fb_flow_export_times", _I, [_P, _P, _U64, _PU64, _P]),
]

_gpu = None


def gpu_lib():
    """Load libflodbadd_gpu.so (raises NativeLibraryMissing if it was not built)."""
    global _gpu
    if _gpu is None:
        if not os.path.exists(GPU_LIB_PATH):
            raise NativeLibraryMissing(
                "%s is missing: run `python -m flodbadd_amd.build` (there is no CPU fallback)" % GPU_LIB_PATH)
        lib = C.CDLL(GPU_LIB_PATH)
        for name, res, args in GPU_SYMBOLS:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.fb_abi_version() != FB_ABI_VERSION:
            raise NativeLibraryMissing("ABI version mismatch")
        _gpu = lib
    return _gpu


def check(rc):
    if rc != FB_OK:
        raise FbError(rc, gpu_lib().fb_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    """ctypes void* of a numpy array's buffer (None for None)."""
    if a is None:
        return None
    return C.c_void_p(a.ctypes.data)


# ---- small device buffer / stream helpers ----------------------------------------------
class DeviceBuffer:
    """Raw device allocation (hipMalloc through the C ABI)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(gpu_lib().fb_dev_alloc(C.byref(p), self.nbytes))
        self.ptr = p

    def upload(self, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes > self.nbytes:
            raise ValueError("upload of %d bytes into a %d-byte device buffer" % (arr.nbytes, self.nbytes))
        check(gpu_lib().fb_memcpy_h2d(self.ptr, ptr(arr), arr.nbytes, stream))
        if stream is None:
            check(gpu_lib().fb_stream_sync(None))
        return self

    def download(self, arr, nbytes=None, stream=None):
        nb = arr.nbytes if nbytes is None else int(nbytes)
        check(gpu_lib().fb_memcpy_d2h(ptr(arr), self.ptr, nb, stream))
        check(gpu_lib().fb_stream_sync(stream))
        return arr

    def memset(self, value=0, stream=None):
        check(gpu_lib().fb_memset_dev(self.ptr, value, self.nbytes, stream))

    def free(self):
        if self.ptr:
            gpu_lib().fb_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host buffer exposed as a numpy uint8 array."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(gpu_lib().fb_host_alloc_pinned(C.byref(p), max(self.nbytes, 1)))
        self.ptr = p
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(p.value))[: self.nbytes]

    def free(self):
        if self.ptr:
            gpu_lib().fb_host_free_pinned(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        p = C.c_void_p()
        check(gpu_lib().fb_stream_create(C.byref(p)))
        self.ptr = p

    def sync(self):
        check(gpu_lib().fb_stream_sync(self.ptr))

    def __del__(self):
        try:
            gpu_lib().fb_stream_destroy(self.ptr)
        except Exception:
            pass


class Event:
    def __init__(self):
        p = C.c_void_p()
        check(gpu_lib().fb_event_create(C.byref(p)))
        self.ptr = p

    def record(self, stream=None):
        check(gpu_lib().fb_event_record(self.ptr, stream.ptr if isinstance(stream, Stream) else stream))

    def wait_spin(self):
        """Poll until the event completed (no blocking wait, no wake-up latency), in C."""
        check(gpu_lib().fb_event_spin(self.ptr))

    def elapsed_ms(self, end):
        ms = C.c_float()
        check(gpu_lib().fb_event_elapsed_ms(C.byref(ms), self.ptr, end.ptr))
        return ms.value

    def __del__(self):
        try:
            gpu_lib().fb_event_destroy(self.ptr)
        except Exception:
            pass


def device_count():
    n = C.c_int(0)
    check(gpu_lib().fb_device_count(C.byref(n)))
    return n.value
