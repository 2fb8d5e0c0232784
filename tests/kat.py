"""Runner for tests/golden/reference_kats.json (known-answer tests transcribed from the
reference's own tests).  A `processor(case_cfg, packets)` returns (records, flows) where
records are the packet-ordered fb_pkt_out SESSION records and flows the fb_flow_rec table."""
import ipaddress
import json
import os

from flodbadd_amd.sessions import (META_DST_SERVICE, Protocol, Session, SessionFilter, SessionPacketData,
                                   flows_to_sessions, histories_from_records)

HERE = os.path.dirname(os.path.abspath(__file__))
KAT_PATH = os.path.join(HERE, "golden", "reference_kats.json")
FLAGS = {"FIN": 0x01, "SYN": 0x02, "RST": 0x04, "PSH": 0x08, "ACK": 0x10}


def load():
    with open(KAT_PATH) as f:
        return json.load(f)


def packets_of(case):
    out = []
    for p in case["packets"]:
        s = Session(Protocol[p["proto"]], ipaddress.ip_address(p["src"]), p["sport"],
                    ipaddress.ip_address(p["dst"]), p["dport"])
        fl = None if p["flags"] is None else sum(FLAGS[x] for x in p["flags"])
        out.append(SessionPacketData(s, p["len"], p["ip_len"], fl))
    return out


def key_of(k):
    return Session(Protocol[k[0]], ipaddress.ip_address(k[1]), k[2], ipaddress.ip_address(k[3]), k[4])


def times_of(case, base_ns=1_700_000_000 * 10**9):
    """Timed cases: the per-packet capture timestamps (ns) of the reference test's sleeps
    (packets[i]["t_ms"] ms after a fixed epoch instant), indexed like the packets; None untimed."""
    if not case.get("timed"):
        return None
    import numpy as np
    return np.array([base_ns + int(round(p["t_ms"] * 1e6)) for p in case["packets"]], dtype=np.uint64)


def check_case(case, records, flows, histories=None, times=None):
    """Assert everything the reference asserts for this case.  The flow table's ordered state
    (hist_len, conn_state) must agree with the history derived from the packet-ordered records;
    `histories` ({table slot: str}, from fb_flow_history_dev) is checked against it too."""
    if case.get("timed") and times is None:
        raise AssertionError("%s: a timed case needs the flows' capture-time records" % case["name"])
    sess = {i.session: i for i in flows_to_sessions(flows, histories=histories, times=times)}
    hist = histories_from_records(records)
    for k, info in sess.items():
        h, cs = hist.get(k, ("", None))
        assert info.stats.hist_len == len(h) and info.stats.conn_state == cs, (case["name"], k, info.stats, h, cs)
        if histories is not None:
            assert info.stats.history == h, (case["name"], k, info.stats.history, h)
    exp = case["expect"]
    name = case["name"]
    if "n_sessions" in exp:
        assert len(sess) == exp["n_sessions"], (name, sorted(sess, key=lambda s: s.sort_key()))
    tol = 1e-9
    for e in exp["sessions"]:
        k = key_of(e["key"])
        assert k in sess, (name, "missing session", k, list(sess))
        st = sess[k].stats
        tol = e.get("tolerance", 1e-9)
        for f in ("outbound_bytes", "inbound_bytes", "orig_pkts", "resp_pkts"):
            if f in e:
                assert getattr(st, f) == e[f], (name, f, getattr(st, f), e[f])
        for f in ("average_packet_size", "inbound_outbound_ratio"):
            if f in e:
                assert abs(getattr(st, f) - e[f]) <= tol, (name, f, getattr(st, f), e[f])
        # segment state (src/packets.rs:137-160, 370-376, 414-420): last_segment_end is Some exactly
        # when a segment has ended, i.e. segment_count > 0
        if "segment_count" in e:
            assert st.segment_count == e["segment_count"], (name, "segment_count", st.segment_count, e["segment_count"])
        if "in_segment" in e:
            assert st.in_segment == e["in_segment"], (name, "in_segment", st.in_segment)
        if "last_segment_end_set" in e:
            assert st.last_segment_end_set == e["last_segment_end_set"], (name, "last_segment_end", st.segment_count)
        if "segment_interarrival_gt" in e:
            assert st.segment_interarrival > e["segment_interarrival_gt"], (name, "interarrival", st.segment_interarrival)
        if "segment_interarrival_ge" in e:
            assert st.segment_interarrival >= e["segment_interarrival_ge"], (name, "interarrival", st.segment_interarrival)
        if "end_time_set" in e:
            assert (st.end_time_ns is not None) == e["end_time_set"], (name, "end_time", st.end_time_ns)
        h, cs = hist.get(k, ("", None))
        if "history" in e:
            assert h == e["history"], (name, h)
        for c in e.get("history_contains", []):
            assert c in h, (name, h, c)
        if "history_order" in e:
            a, b = e["history_order"]
            assert h.index(a) < h.index(b), (name, h)
        if e.get("conn_state_set"):
            assert cs is not None, (name, h)
        if "dst_service" in e:
            # dst_service is set at session creation from the first packet (src/packets.rs:441-464)
            first = next(r for r in records if Session.from_key(r) == k)
            assert bool(int(first["meta"]) & META_DST_SERVICE) == e["dst_service"], (name, k.dst_port)
            # ... and stored in the session (SessionInfo.dst_service.is_some(), src/packets.rs:866-870)
            assert (sess[k].dst_service is not None) == e["dst_service"], (name, sess[k].dst_service)


def filter_of(case):
    return SessionFilter[case["filter"]]
