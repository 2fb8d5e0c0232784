"""ctypes wrapper of oracle/liboracle.so (the C restatement).  TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
ROOT = os.path.dirname(HERE)
BITMAP_PATH = os.path.join(ROOT, "flodbadd_amd", "data", "service_ports.bin")

# Record layouts are defined once, in the product's binding of include/flodbadd_gpu.h.
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd._native import (DNS_OUT_DTYPE, FB_IP_DTYPE, FLOW_REC_DTYPE, LAN_V6_DTYPE, PARSED_DTYPE,  # noqa: E402
                                  PKT_OUT_DTYPE, STATS_DTYPE)


class LanV6(C.Structure):
    _fields_ = [("net", C.c_uint32 * 4), ("prefix", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class FbIp(C.Structure):
    _fields_ = [("addr", C.c_uint32 * 4), ("family", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class OrcCfg(C.Structure):
    _fields_ = [("filter", C.c_uint32), ("service_bitmap", C.c_uint8 * 8192), ("n_lan_v6", C.c_uint32),
                ("lan_v6", LanV6 * 64), ("n_own_ips", C.c_uint32), ("own_ips", FbIp * 64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("%s missing: run `python -m flodbadd_amd.build`" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        P, U32, U64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.orc_parse_classify.restype = C.c_int
        L.orc_parse_classify.argtypes = [P, P, U64, P, U32, P, C.POINTER(U32), P, C.POINTER(U32), P, P]
        L.orc_process_parsed.restype = C.c_int
        L.orc_process_parsed.argtypes = [P, P, U32, P, C.POINTER(U32), P, P]
        L.orc_asn_prepare.restype = C.c_uint32
        L.orc_asn_prepare.argtypes = [P, C.c_uint32, C.c_uint32]
        L.orc_asn_lookup.restype = C.c_int32
        L.orc_asn_lookup.argtypes = [P, C.c_uint32, C.c_uint32, P]
        L.orc_blacklist_mask.restype = U64
        L.orc_blacklist_mask.argtypes = [P, C.c_uint32, C.c_uint32, P]
        L.orc_enrich_keys.argtypes = [P, P, C.c_uint32, P, C.c_uint32, P, C.c_uint32, P, C.c_uint32, P]
        L.orc_parse_classify_mt.argtypes = [P, P, U64, P, U32, P, P, P, P, P, C.c_int]
        L.orc_dns_parse.restype = C.c_uint32
        L.orc_dns_parse.argtypes = [P, C.c_uint32, C.c_uint32, P, C.c_char_p, P]
        L.orc_flows_new.restype = P
        L.orc_flows_free.argtypes = [P]
        L.orc_flows_clear.argtypes = [P]
        L.orc_flows_update.argtypes = [P, P, U64, P]
        L.orc_flows_update_timed.argtypes = [P, P, U64, P, P]
        L.orc_flows_export_times.restype = U64
        L.orc_flows_export_times.argtypes = [P, P, P, U64]
        L.orc_flows_count.restype = U64
        L.orc_flows_count.argtypes = [P]
        L.orc_flows_export_sorted.restype = U64
        L.orc_flows_export_sorted.argtypes = [P, P, U64]
        L.orc_flows_history.restype = C.c_int64
        L.orc_flows_history.argtypes = [P, P, C.c_char_p, U64, C.c_char_p, U64]
        L.orc_pipeline.restype = U64
        L.orc_pipeline.argtypes = [P, P, P, U64, P, U32, P, P]
        L.orc_pipeline_mt.restype = U64
        L.orc_pipeline_mt.argtypes = [P, P, C.c_int, P, U64, P, U32, P, P, P]
        L.orc_key_cmp.restype = C.c_int
        L.orc_key_cmp.argtypes = [P, P]
        L.orc_flow_hash.restype = U64
        L.orc_flow_hash.argtypes = [P]
        L.orc_flows_export_merge.restype = U64
        L.orc_flows_export_merge.argtypes = [P, U32, U32, U64, P, P]
        L.orc_flows_export_merge_map.restype = U64
        L.orc_flows_export_merge_map.argtypes = [P, U32, U32, P, P, P]
        L.orc_flow_merge.restype = U64
        L.orc_flow_merge.argtypes = [P, U64, P]
        _lib = L
    return _lib


def default_bitmap():
    with open(BITMAP_PATH, "rb") as f:
        return f.read()


def make_cfg(session_filter=2, bitmap=None, lan_v6=None, own_ips=None):
    """lan_v6 / own_ips are LAN_V6_DTYPE / FB_IP_DTYPE arrays (see flodbadd_amd.capture)."""
    c = OrcCfg()
    c.filter = int(session_filter)
    bm = default_bitmap() if bitmap is None else bytes(bitmap)
    C.memmove(c.service_bitmap, bm, 8192)
    if lan_v6 is not None and len(lan_v6):
        lan_v6 = np.ascontiguousarray(lan_v6, dtype=LAN_V6_DTYPE)
        c.n_lan_v6 = len(lan_v6)
        C.memmove(C.addressof(c.lan_v6), lan_v6.ctypes.data, lan_v6.nbytes)
    if own_ips is not None and len(own_ips):
        own_ips = np.ascontiguousarray(own_ips, dtype=FB_IP_DTYPE)
        c.n_own_ips = len(own_ips)
        C.memmove(C.addressof(c.own_ips), own_ips.ctypes.data, own_ips.nbytes)
    return c


def parse_classify(cfg, frames, offsets):
    """Returns (records, dns, cls, stats) exactly as fb_parse_classify would."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    n = offsets.size - 1
    out = np.zeros(max(n, 1), dtype=PKT_OUT_DTYPE)
    dns = np.zeros(max(n, 1), dtype=DNS_OUT_DTYPE)
    cls = np.zeros(max(n, 1), dtype=np.uint8)
    st = np.zeros(1, dtype=STATS_DTYPE)
    no, nd = C.c_uint32(), C.c_uint32()
    lib().orc_parse_classify(C.byref(cfg), frames.ctypes.data, frames.nbytes, offsets.ctypes.data, n,
                             out.ctypes.data, C.byref(no), dns.ctypes.data, C.byref(nd), cls.ctypes.data,
                             st.ctypes.data)
    return out[: no.value], dns[: nd.value], cls[:n], st


def process_parsed(cfg, parsed):
    """Batched process_parsed_packet over PARSED_DTYPE records -> (records, cls, stats)."""
    parsed = np.ascontiguousarray(parsed, dtype=PARSED_DTYPE)
    n = parsed.size
    out = np.zeros(max(n, 1), dtype=PKT_OUT_DTYPE)
    cls = np.zeros(max(n, 1), dtype=np.uint8)
    st = np.zeros(1, dtype=STATS_DTYPE)
    no = C.c_uint32()
    lib().orc_process_parsed(C.byref(cfg), parsed.ctypes.data if n else None, n, out.ctypes.data, C.byref(no),
                             cls.ctypes.data, st.ctypes.data)
    return out[: no.value], cls[:n], st


def asn_prepare(table, family):
    """Db::from_tsv's filter + stable sort of one family's ASN_RANGE_DTYPE table (a copy)."""
    t = np.ascontiguousarray(table, dtype=N.ASN_RANGE_DTYPE).copy()
    m = lib().orc_asn_prepare(t.ctypes.data if len(t) else None, len(t), family)
    return t[:m]


def enrich_keys(cfg, a4, a6, cidrs, keys):
    """orc_enrich_keys over 40-B keys (any record array whose first 40 bytes are the key);
    a4/a6 already through asn_prepare."""
    kb = np.ascontiguousarray(np.frombuffer(b"".join(k.tobytes()[:40] for k in keys), dtype=np.uint8))
    n = len(keys)
    out = np.zeros(max(n, 1), dtype=N.FLOW_ENRICH_DTYPE)
    a4 = np.ascontiguousarray(a4, dtype=N.ASN_RANGE_DTYPE)
    a6 = np.ascontiguousarray(a6, dtype=N.ASN_RANGE_DTYPE)
    cidrs = np.ascontiguousarray(cidrs, dtype=N.CIDR_DTYPE)
    lib().orc_enrich_keys(C.byref(cfg), a4.ctypes.data if len(a4) else None, len(a4),
                          a6.ctypes.data if len(a6) else None, len(a6), cidrs.ctypes.data if len(cidrs) else None,
                          len(cidrs), kb.ctypes.data if n else None, n, out.ctypes.data)
    return out[:n]


def ip_lookup(a4, a6, cidrs, ips):
    """Db::lookup + the blacklist scan for addresses -> (int32 records, uint64 masks)."""
    from flodbadd_amd.sessions import ip_to_words
    a4 = np.ascontiguousarray(a4, dtype=N.ASN_RANGE_DTYPE)
    a6 = np.ascontiguousarray(a6, dtype=N.ASN_RANGE_DTYPE)
    cidrs = np.ascontiguousarray(cidrs, dtype=N.CIDR_DTYPE)
    asn, lists = [], []
    for ip in ips:
        w, fam = ip_to_words(ip)
        w = np.ascontiguousarray(w, dtype=np.uint32)
        t = a6 if fam == 10 else a4
        asn.append(lib().orc_asn_lookup(t.ctypes.data if len(t) else None, len(t), fam, w.ctypes.data))
        lists.append(lib().orc_blacklist_mask(cidrs.ctypes.data if len(cidrs) else None, len(cidrs), fam,
                                              w.ctypes.data))
    return np.array(asn, dtype=np.int32), np.array(lists, dtype=np.uint64)


def dns_parse(payload, pkt_index=0):
    """orc_dns_parse -> (DNS_MSG_DTYPE record, name bytes, [fb_ip addrs])."""
    pl = np.frombuffer(bytes(payload), dtype=np.uint8).copy()
    r = np.zeros(1, dtype=N.DNS_MSG_DTYPE)
    name = C.create_string_buffer(N.FB_DNS_MAX_NAME)
    addrs = np.zeros(N.FB_DNS_MAX_ADDRS, dtype=FB_IP_DTYPE)
    lib().orc_dns_parse(pl.ctypes.data if pl.size else None, pl.size, pkt_index, r.ctypes.data, name,
                        addrs.ctypes.data)
    return r[0], name.raw[: int(r[0]["name_len"])], addrs[: int(r[0]["n_addrs"])]


class Flows:
    """The oracle's session table (DashMap restatement)."""

    def __init__(self):
        self.h = C.c_void_p(lib().orc_flows_new())

    def update(self, recs, stats=None, ts=None):
        """One update call.  ts (timed tables): the batch's per-frame capture timestamps (uint64 ns,
        indexed by pkt_index)."""
        recs = np.ascontiguousarray(recs, dtype=PKT_OUT_DTYPE)
        if ts is None:
            lib().orc_flows_update(self.h, recs.ctypes.data if recs.size else None, recs.size,
                                   stats.ctypes.data if stats is not None else None)
        else:
            ts = np.ascontiguousarray(ts, dtype=np.uint64)
            lib().orc_flows_update_timed(self.h, recs.ctypes.data if recs.size else None, recs.size,
                                         stats.ctypes.data if stats is not None else None,
                                         ts.ctypes.data if ts.size else None)
        self._keep = ts

    def export_times(self, with_ref=False):
        """FLOW_TIME_DTYPE per flow in export_sorted order; with_ref: also the reference's own f64
        (total_segment_interarrival, segment_interarrival) per flow, [F, 2]."""
        from flodbadd_amd._native import FLOW_TIME_DTYPE
        n = self.count()
        out = np.zeros(max(n, 1), dtype=FLOW_TIME_DTYPE)
        ref = np.zeros((max(n, 1), 2), dtype=np.float64)
        m = lib().orc_flows_export_times(self.h, out.ctypes.data, ref.ctypes.data, n)
        return (out[:m], ref[:m]) if with_ref else out[:m]

    def count(self):
        return lib().orc_flows_count(self.h)

    def export_sorted(self):
        n = self.count()
        out = np.zeros(max(n, 1), dtype=FLOW_REC_DTYPE)
        m = lib().orc_flows_export_sorted(self.h, out.ctypes.data, n)
        return out[:m]

    def history(self, key_rec):
        """key_rec: a PKT_OUT_DTYPE or FLOW_REC_DTYPE element (uses its first 40 bytes)."""
        kb = np.frombuffer(key_rec.tobytes()[:40], dtype=np.uint8).copy()
        if not hasattr(self, "_buf"):
            self._buf, self._cs = C.create_string_buffer(1 << 16), C.create_string_buffer(8)
        n = lib().orc_flows_history(self.h, kb.ctypes.data, self._buf, len(self._buf), self._cs, 8)
        if n > len(self._buf):
            self._buf = C.create_string_buffer(int(n))
            n = lib().orc_flows_history(self.h, kb.ctypes.data, self._buf, len(self._buf), self._cs, 8)
        if n < 0:
            return None, None
        return self._buf.raw[:n].decode(), (self._cs.value.decode() or None)

    def export_merge(self, world, rank, shard_first=0, call_map=None):
        """orc_flows_export_merge (orc_flows_export_merge_map with `call_map`, a sequence of
        global batch << 32 | shard start per update call): FLOW_MREC_DTYPE records grouped by owner
        rank, and the group sizes."""
        n = self.count()
        out = np.zeros(max(n, 1), dtype=N.FLOW_MREC_DTYPE)
        counts = np.zeros(world, dtype=np.uint64)
        if call_map is None:
            m = lib().orc_flows_export_merge(self.h, world, rank, shard_first, out.ctypes.data, counts.ctypes.data)
        else:
            cm = np.ascontiguousarray(np.asarray(call_map, dtype=np.uint64).reshape(-1))
            if cm.size == 0:
                cm = np.zeros(1, dtype=np.uint64)
            m = lib().orc_flows_export_merge_map(self.h, world, rank, cm.ctypes.data, out.ctypes.data,
                                                 counts.ctypes.data)
        return out[:m], counts

    def clear(self):
        lib().orc_flows_clear(self.h)

    def __del__(self):
        try:
            lib().orc_flows_free(self.h)
        except Exception:
            pass


def pipeline_mt(cfg, frames, offsets, threads, tables=None):
    """orc_pipeline_mt: all-cores parse + classify + session upsert.  Returns (per-thread Flows,
    stats); the union of the tables equals the single-thread table."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    n = offsets.size - 1
    tables = tables or [Flows() for _ in range(threads)]
    hs = (C.c_void_p * threads)(*[t.h.value for t in tables])
    out = np.zeros(max(n, 1), dtype=PKT_OUT_DTYPE)
    dns = np.zeros(max(n, 1), dtype=DNS_OUT_DTYPE)
    st = np.zeros(1, dtype=STATS_DTYPE)
    lib().orc_pipeline_mt(C.byref(cfg), hs, threads, frames.ctypes.data, frames.nbytes, offsets.ctypes.data, n,
                          out.ctypes.data, dns.ctypes.data, st.ctypes.data)
    return tables, st


def flow_merge(mrecs):
    """orc_flow_merge: one owner's received FLOW_MREC_DTYPE records -> merged FLOW_REC_DTYPE records."""
    mrecs = np.ascontiguousarray(mrecs, dtype=N.FLOW_MREC_DTYPE)
    out = np.zeros(max(len(mrecs), 1), dtype=FLOW_REC_DTYPE)
    k = lib().orc_flow_merge(mrecs.ctypes.data if len(mrecs) else None, len(mrecs), out.ctypes.data)
    return out[:k]
