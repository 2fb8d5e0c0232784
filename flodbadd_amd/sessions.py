"""Host-side session model, mirroring the reference's types (src/sessions.rs).

Only data-model plumbing lives here: converting between the C-ABI `fb_session_key` layout and
Session objects, derived statistics computed from integer counters, and the post-hoc
bucket split `filter_sessions` (src/sessions.rs:678-692), which in the reference runs per
query over the session list, not per packet.  Per-packet work never runs here.
"""
import enum
import ipaddress
import json
import os

import numpy as np
from dataclasses import dataclass, field
from typing import List, Optional

from ._native import (CONN_STATES, FB_FILTER_ALL, FB_FILTER_GLOBAL_ONLY, FB_FILTER_LOCAL_ONLY, FB_SEEN_NONE,
                      FLOW_REC_DTYPE, SESSION_DST_SERVICE, SESSION_LOCAL_DST, SESSION_LOCAL_SRC, SESSION_SELF_DST,
                      SESSION_SELF_SRC,
                      META_DST_SERVICE, META_HAS_FLAGS, META_LOCAL_DST, META_LOCAL_SRC, META_ORIGINATOR,
                      META_SELF_DST, META_SELF_SRC, META_SWAP, PARSED_DTYPE, PKT_OUT_DTYPE)


class Protocol(enum.IntEnum):
    """src/sessions.rs:17-21 (derived Ord: TCP < UDP)."""
    TCP = 6
    UDP = 17


class SessionFilter(enum.IntEnum):
    """src/sessions.rs:173-178 (same discriminant order)."""
    LocalOnly = FB_FILTER_LOCAL_ONLY
    GlobalOnly = FB_FILTER_GLOBAL_ONLY
    All = FB_FILTER_ALL


def ip_to_words(ip):
    """session_to_key word format (src/l7_ebpf.rs:78-104): v4 numeric in word 0; v6 4 BE words."""
    ip = ipaddress.ip_address(ip)
    if ip.version == 4:
        return (int(ip), 0, 0, 0), 2
    v = int(ip)
    return tuple((v >> (96 - 32 * k)) & 0xFFFFFFFF for k in range(4)), 10


def words_to_ip(words, family):
    if family == 2:
        return ipaddress.IPv4Address(int(words[0]))
    v = 0
    for w in words:
        v = (v << 32) | int(w)
    return ipaddress.IPv6Address(v)


@dataclass(frozen=True, order=False)
class Session:
    """The 5-tuple key, src/sessions.rs:23-30."""
    protocol: Protocol
    src_ip: object
    src_port: int
    dst_ip: object
    dst_port: int

    def sort_key(self):
        """Derived Ord: protocol, src_ip (V4 < V6, then octets), src_port, dst_ip, dst_port."""
        return (int(self.protocol), self.src_ip.version, int(self.src_ip), self.src_port,
                self.dst_ip.version, int(self.dst_ip), self.dst_port)

    def __lt__(self, other):
        return self.sort_key() < other.sort_key()

    def reversed(self):
        return Session(self.protocol, self.dst_ip, self.dst_port, self.src_ip, self.src_port)

    @staticmethod
    def from_key(rec):
        fam = int(rec["family"])
        return Session(Protocol(int(rec["protocol"])), words_to_ip(rec["src_ip"], fam), int(rec["src_port"]),
                       words_to_ip(rec["dst_ip"], fam), int(rec["dst_port"]))

    def key_fields(self):
        s, fam = ip_to_words(self.src_ip)
        d, _ = ip_to_words(self.dst_ip)
        return s, d, fam


@dataclass
class SessionPacketData:
    """src/packets.rs:91-98 (per emitted record; raw session = key reversed when swapped)."""
    session: Session
    packet_length: int
    ip_packet_length: int
    flags: Optional[int]


@dataclass
class SessionStats:
    """Integer counters of src/sessions.rs:73-96 + the two derived f64s
    (src/packets.rs:122-135), recomputed from the final counters."""
    inbound_bytes: int = 0
    outbound_bytes: int = 0
    orig_pkts: int = 0
    resp_pkts: int = 0
    orig_ip_bytes: int = 0
    resp_ip_bytes: int = 0
    history: str = ""
    conn_state: Optional[str] = None
    # positions ((flow update call << 32) | pkt_index) standing for start_time / last_activity /
    # end_time (src/sessions.rs:74-76); end None until the first FIN/RST
    first_seen: int = 0
    last_seen: int = 0
    end_seen: Optional[int] = None
    hist_len: int = 0
    # segment detection (src/sessions.rs:88-93; src/packets.rs:137-160, 370-376, 414-420) under the
    # no-timeout model: TCP packets with PSH counted, in a segment unless the latest packet had PSH
    segment_count: int = 0
    in_segment: bool = False
    # timed contexts (fb_flow_time, FB_CFG_TIMED): capture times in ns since the epoch (the
    # reference's DateTime<Utc> start_time / last_activity / end_time / current_segment_start /
    # last_segment_end, src/sessions.rs:74-92) and the exact interarrival sum in ms; None untimed
    start_time_ns: Optional[int] = None
    last_activity_ns: Optional[int] = None
    end_time_ns: Optional[int] = None
    current_segment_start_ns: Optional[int] = None
    last_segment_end_ns: Optional[int] = None
    total_segment_interarrival_ms: int = 0
    segment_interarrival_div: int = 0
    segment_timeout: float = 5.0  # src/packets.rs:379

    @property
    def total_segment_interarrival(self):
        """Seconds (f64), as src/packets.rs:166 accumulates it (from the exact integer ms sum)."""
        return self.total_segment_interarrival_ms / 1000.0

    @property
    def segment_interarrival(self):
        """src/packets.rs:167-171: the total over segment_count - 1 at the last accepted term."""
        d = self.segment_interarrival_div
        return self.total_segment_interarrival / d if d > 0 else 0.0

    @property
    def last_segment_end_set(self):
        """last_segment_end.is_some(): timed, from the capture times; untimed, a segment has ended."""
        if self.start_time_ns is not None:
            return self.last_segment_end_ns is not None
        return self.segment_count > 0

    @property
    def average_packet_size(self):
        tp = self.orig_pkts + self.resp_pkts
        return (self.inbound_bytes + self.outbound_bytes) / tp if tp > 0 else 0.0

    @property
    def inbound_outbound_ratio(self):
        return self.inbound_bytes / self.outbound_bytes if self.outbound_bytes > 0 else 0.0


@dataclass
class SessionInfo:
    """Subset of src/sessions.rs:40-61 that the GPU path owns.  is_local_* / is_self_* and
    dst_service are the values stored when the session was inserted (src/packets.rs:429-466,
    fb_flow_rec.session_flags)."""
    session: Session
    stats: SessionStats = field(default_factory=SessionStats)
    is_local_src: bool = False
    is_local_dst: bool = False
    is_self_src: bool = False
    is_self_dst: bool = False
    dst_service: Optional[str] = None


_SERVICE_NAMES = None


def service_name(port):
    """get_name_from_port (src/port_vulns.rs:213-228) over the reference's built-in port table
    (data/service_names.json, generated by tools/gen_service_bitmap.py with the service bitmap):
    the name, or "" for a port the table does not name."""
    global _SERVICE_NAMES
    if _SERVICE_NAMES is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "service_names.json")) as f:
            _SERVICE_NAMES = {int(k): v for k, v in json.load(f).items()}
    return _SERVICE_NAMES.get(int(port), "")


def is_lan_ip(ip, lan_v6=()):
    """is_lan_ip, src/ip.rs:199-242: the IPv4 fast check (ip.rs:55-91), the IPv6 special ranges
    (ip.rs:112-136) and the interface prefixes of the LAN cache (ip.rs:141-156, 164-191), given as
    [(address, prefix_len)] like FlodbaddGpuCapture's lan_v6.  Host-side: the reference evaluates it
    per query in is_local_session! / filter_sessions (src/sessions.rs:660-692)."""
    ip = ipaddress.ip_address(ip)
    if ip.version == 4:
        v = int(ip)
        return (v in (0, 0xFFFFFFFF) or (v >> 24) in (127, 10) or (v >> 28) == 0xE or (v >> 16) in (0xA9FE, 0xC0A8)
                or ((v >> 24) == 172 and 16 <= ((v >> 16) & 0xFF) <= 31))
    v = int(ip)
    s0 = v >> 112
    if v in (0, 1) or (s0 & 0xFFC0) == 0xFE80 or (s0 & 0xFF00) == 0xFF00 or (s0 & 0xFE00) == 0xFC00:
        return True
    for net, pfx in lan_v6:
        mask = 0 if pfx == 0 else ((1 << 128) - 1) ^ ((1 << (128 - pfx)) - 1)
        if (v & mask) == (int(ipaddress.IPv6Address(net)) & mask):
            return True
    return False


def is_local_session(info, lan_v6=()):
    """is_local_session! (src/sessions.rs:660-666): both key addresses LAN, evaluated now."""
    return is_lan_ip(info.session.src_ip, lan_v6) and is_lan_ip(info.session.dst_ip, lan_v6)


def records_to_packets(recs):
    """fb_pkt_out records -> SessionPacketData (raw direction restored from the SWAP bit)."""
    if recs.dtype != PKT_OUT_DTYPE:
        raise TypeError("expected fb_pkt_out records (PKT_OUT_DTYPE), got %s" % recs.dtype)
    out = []
    for r in recs:
        key = Session.from_key(r)
        raw = key.reversed() if int(r["meta"]) & META_SWAP else key
        flags = int(r["tcp_flags"]) if int(r["meta"]) & META_HAS_FLAGS else None
        out.append(SessionPacketData(raw, int(r["packet_length"]), int(r["ip_packet_length"]), flags))
    return out


def packets_to_parsed(packets):
    """SessionPacketData list -> PARSED_DTYPE array (fb_parsed_pkt), pkt_index = list position."""
    a = np.zeros(len(packets), dtype=PARSED_DTYPE)
    for i, p in enumerate(packets):
        s, d, fam = p.session.key_fields()
        a[i]["src_ip"], a[i]["dst_ip"] = s, d
        a[i]["src_port"], a[i]["dst_port"] = p.session.src_port, p.session.dst_port
        a[i]["protocol"], a[i]["family"] = int(p.session.protocol), fam
        a[i]["packet_length"], a[i]["ip_packet_length"] = p.packet_length, p.ip_packet_length
        a[i]["tcp_flags"] = p.flags or 0
        a[i]["has_flags"] = 0 if p.flags is None else 1
        a[i]["pkt_index"] = i
    return a


def determine_conn_state(history):
    """src/packets.rs:539-559."""
    h = set(history)
    if {"S", "H", "F", "f"} <= h:
        return "SF"
    if "S" in h and "h" not in h and "r" not in h:
        return "S0"
    if "R" in h or "r" in h:
        return "REJ"
    if "S" in h and "H" in h and "F" not in h and "f" not in h:
        return "S1"
    return "-"


def histories_from_records(recs):
    """Per-flow history strings + conn_state from packet-ordered fb_pkt_out records.

    The GPU emits each packet's map_tcp_flags char (src/packets.rs:561-601) in its record; the
    ordered per-flow string (src/packets.rs:187-198, 410-426) is the concatenation in packet order,
    and conn_state is fixed at the first FIN/RST.  Returns {Session: (history, conn_state)}."""
    if recs.dtype != PKT_OUT_DTYPE:
        raise TypeError("expected fb_pkt_out records (PKT_OUT_DTYPE), got %s" % recs.dtype)
    hist, state = {}, {}
    for r in recs[np.argsort(recs["pkt_index"], kind="stable")]:
        if not int(r["meta"]) & META_HAS_FLAGS:
            continue
        k = Session.from_key(r)
        h = hist.get(k, "") + chr(int(r["hist_char"]))
        hist[k] = h
        if int(r["tcp_flags"]) & 0x05 and k not in state:  # FIN | RST
            state[k] = determine_conn_state(h)
    return {k: (h, state.get(k)) for k, h in hist.items()}


def flows_to_sessions(flows, histories=None, times=None):
    """fb_flow_rec records -> SessionInfo list sorted by the derived Ord of Session.  `histories`
    ({table slot: str}, FlodbaddGpuCapture.histories) supplies the history strings; the locality
    flags and dst_service come from fb_flow_rec.session_flags (stored at insert, src/packets.rs:
    429-466; dst_service = the key's dst port name, or its number for a port only a service table
    set at run time names).  `times` (timed contexts): FLOW_TIME_DTYPE records, either joined by
    table slot (fb_flow_export_times) or, when every slot field is 0, one per flow in `flows` order."""
    if flows.dtype != FLOW_REC_DTYPE:
        raise TypeError("expected fb_flow_rec records (FLOW_REC_DTYPE), got %s" % flows.dtype)
    tmap = None
    if times is not None:
        if len(times) == len(flows) and (len(times) == 0 or not times["slot"].any()):
            tmap = {i: t for i, t in enumerate(times)}
        else:
            tmap = {int(t["slot"]): t for t in times}
    out = []
    for idx, r in enumerate(flows):
        end = int(r["end_seen"])
        st = SessionStats(int(r["inbound_bytes"]), int(r["outbound_bytes"]), int(r["orig_pkts"]),
                          int(r["resp_pkts"]), int(r["orig_ip_bytes"]), int(r["resp_ip_bytes"]),
                          histories.get(int(r["slot"]), "") if histories is not None else "",
                          CONN_STATES[int(r["conn_state"])], int(r["first_seen"]), int(r["last_seen"]),
                          None if end == FB_SEEN_NONE else end, int(r["hist_len"]), int(r["segment_count"]),
                          bool(r["in_segment"]))
        if tmap is not None:
            t = tmap[idx] if (len(times) == len(flows) and (len(times) == 0 or not times["slot"].any())) \
                else tmap[int(r["slot"])]
            none = lambda v: None if int(v) == FB_SEEN_NONE else int(v)  # noqa: E731
            st.start_time_ns, st.last_activity_ns = int(t["start_time_ns"]), int(t["last_activity_ns"])
            st.end_time_ns, st.last_segment_end_ns = none(t["end_time_ns"]), none(t["last_segment_end_ns"])
            st.current_segment_start_ns = int(t["current_segment_start_ns"])
            st.total_segment_interarrival_ms = int(t["total_segment_interarrival_ms"])
            st.segment_interarrival_div = int(t["segment_interarrival_div"])
        s = Session.from_key(r)
        f = int(r["session_flags"])
        svc = (service_name(s.dst_port) or str(s.dst_port)) if f & SESSION_DST_SERVICE else None
        info = SessionInfo(s, st, bool(f & SESSION_LOCAL_SRC), bool(f & SESSION_LOCAL_DST),
                           bool(f & SESSION_SELF_SRC), bool(f & SESSION_SELF_DST), svc)
        out.append(info)
    out.sort(key=lambda i: i.session.sort_key())
    return out


def filter_sessions(sessions: List[SessionInfo], flt: SessionFilter, lan_v6=()) -> List[SessionInfo]:
    """src/sessions.rs:678-692: is_local_session! / is_global_session! evaluate is_lan_ip on the
    session's addresses at call time (src/sessions.rs:660-672), not the flags stored at insert."""
    if flt == SessionFilter.LocalOnly:
        return [s for s in sessions if is_local_session(s, lan_v6)]
    if flt == SessionFilter.GlobalOnly:
        return [s for s in sessions if not is_local_session(s, lan_v6)]
    return list(sessions)


__all__ = ["Protocol", "SessionFilter", "Session", "SessionPacketData", "SessionStats", "SessionInfo",
           "ip_to_words", "words_to_ip", "service_name", "records_to_packets", "flows_to_sessions", "filter_sessions",
           "packets_to_parsed", "determine_conn_state", "histories_from_records", "is_lan_ip", "is_local_session",
           "META_HAS_FLAGS", "META_SWAP", "META_ORIGINATOR", "META_LOCAL_SRC", "META_LOCAL_DST",
           "META_SELF_SRC", "META_SELF_DST", "META_DST_SERVICE"]
