"""The CPU oracle against the reference's own known-answer tests and fixtures:
transcribed process_parsed_packet KATs, the is_lan_ip vectors, the service-port table digest.
This pins the oracle before it is trusted as the checker of the GPU path."""
import hashlib

import numpy as np
import pytest

import kat
from flodbadd_amd import _native as N
from flodbadd_amd.capture import lan_v6_table, own_ip_table
from flodbadd_amd.sessions import SessionFilter, ip_to_words, packets_to_parsed
from oracle import coracle, pyoracle

KATS = kat.load()


def oracle_process(case):
    cfg = coracle.make_cfg(int(kat.filter_of(case)), own_ips=own_ip_table(case["own_ips"]))
    recs, cls, st = coracle.process_parsed(cfg, packets_to_parsed(kat.packets_of(case)))
    flows = coracle.Flows()
    fst = np.zeros(1, dtype=N.STATS_DTYPE)
    flows.update(recs, fst, ts=kat.times_of(case))
    return recs, flows, st


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_oracle_reference_kat(case):
    recs, flows, st = oracle_process(case)
    kat.check_case(case, recs, flows.export_sorted(), times=flows.export_times() if case.get("timed") else None)
    # PACKET_STATS counts every packet before the filter (src/packets.rs:211-227)
    assert int(st[0]["total_processed"]) == len(case["packets"])


TIMED = [c for c in KATS["cases"] if c.get("timed")]


def test_timed_cases_present():
    """The clock-dependent asserts are transcribed: the >= 5 s gap (TCP and UDP) and the interarrival."""
    names = {c["name"] for c in TIMED}
    assert {"test_packet_statistics/timed_final", "test_udp_segment_timeout/timed_after_pkt2"} <= names
    final = next(c for c in TIMED if c["name"] == "test_packet_statistics/timed_final")
    assert final["expect"]["sessions"][0]["segment_count"] == 2


@pytest.mark.parametrize("case", TIMED, ids=[c["name"] for c in TIMED])
def test_timed_kat_c_oracle_equals_python_oracle(case):
    """The C restatement's capture-time state equals the independent Python restatement's
    (pyoracle.SessionTable with `now`), field by field -- and its exact integer interarrival sum in
    ms / 1000 equals the reference's own f64 running sum (both restatements keep it) to 1e-12 s."""
    from flodbadd_amd.sessions import Session
    recs, flows, _ = oracle_process(case)
    ts = kat.times_of(case)
    t, ref = flows.export_times(with_ref=True)
    fr = flows.export_sorted()
    table = pyoracle.SessionTable()
    for i, p in enumerate(kat.packets_of(case)):
        pc = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=int(kat.filter_of(case)),
                                         own_ips=case["own_ips"])
        import ipaddress
        c = pyoracle.classify(pc, ("tcp" if int(p.session.protocol) == 6 else "udp", int(p.session.protocol),
                                   p.session.src_ip, p.session.src_port, p.session.dst_ip, p.session.dst_port,
                                   p.packet_length, p.ip_packet_length, p.flags))
        if c["klass"] != "filtered":
            table.process(c, int(ts[i]))
    py = pyoracle.table_times(table)
    none = lambda v: None if int(v) == N.FB_SEEN_NONE else int(v)  # noqa: E731
    for r, x, (rt, ri) in zip(fr, t, ref):
        k = Session.from_key(r)
        e = py[(int(k.protocol), k.src_ip, k.src_port, k.dst_ip, k.dst_port)]
        got = (int(x["start_time_ns"]), int(x["last_activity_ns"]), none(x["end_time_ns"]),
               int(x["current_segment_start_ns"]), none(x["last_segment_end_ns"]),
               int(x["total_segment_interarrival_ms"]), e[6], int(x["segment_interarrival_div"]),
               int(x["segment_count"]), bool(x["in_segment"]))
        assert got == e, (case["name"], got, e)
        assert abs(rt - e[6]) <= 1e-12 and abs(int(x["total_segment_interarrival_ms"]) / 1000.0 - rt) <= 1e-12


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_oracle_history_matches_flow_table(case):
    """The per-packet history chars, concatenated in packet order, equal the oracle session
    table's own ordered history (the form the GPU path uses for history)."""
    from flodbadd_amd.sessions import histories_from_records
    recs, flows, _ = oracle_process(case)
    for k, (h, cs) in histories_from_records(recs).items():
        rec = np.zeros(1, dtype=N.PKT_OUT_DTYPE)
        s, d, fam = k.key_fields()
        rec[0]["src_ip"], rec[0]["dst_ip"], rec[0]["family"] = s, d, fam
        rec[0]["src_port"], rec[0]["dst_port"], rec[0]["protocol"] = k.src_port, k.dst_port, int(k.protocol)
        oh, ocs = flows.history(rec[0])
        assert (oh, ocs) == (h, cs)


def test_service_bitmap_digest_and_named_ports():
    sb = KATS["service_bitmap"]
    bm = coracle.default_bitmap()
    assert hashlib.sha256(bm).hexdigest() == sb["sha256"]
    named = lambda p: bool(bm[p >> 3] & (1 << (p & 7)))  # noqa: E731
    assert all(named(p) for p in sb["named"])
    assert not any(named(p) for p in sb["unnamed"])


def _lan_through_filter(ip, lan_v6):
    """is_lan_ip(ip) observed through the product contract: a src==dst packet is local iff
    is_lan(ip) (is_local_session!, src/sessions.rs:660-672), so LocalOnly keeps it iff LAN."""
    from flodbadd_amd.sessions import Protocol, Session, SessionPacketData
    import ipaddress
    a = ipaddress.ip_address(ip)
    pk = SessionPacketData(Session(Protocol.UDP, a, 40001, a, 40002), 10, 38, None)
    cfg = coracle.make_cfg(int(SessionFilter.LocalOnly), lan_v6=lan_v6_table(lan_v6))
    recs, cls, st = coracle.process_parsed(cfg, packets_to_parsed([pk]))
    return int(cls[0]) == N.FB_CLASS_SESSION


def test_is_lan_ip_reference_vectors():
    lan = KATS["lan"]
    for ip, expect in lan["vectors"]:
        assert _lan_through_filter(ip, lan["lan_v6_prefixes"]) == expect, ip
        # the independent Python restatement agrees
        pc = pyoracle.Config(lan_v6=lan["lan_v6_prefixes"])
        import ipaddress
        assert pc.is_lan(ipaddress.ip_address(ip)) == expect, ip


def test_ip_words_layout():
    """session_to_key (src/l7_ebpf.rs:78-104): v4 numeric in word 0, v6 big-endian words."""
    assert ip_to_words("192.168.1.1") == ((0xC0A80101, 0, 0, 0), 2)
    assert ip_to_words("2001:db8::1") == ((0x20010DB8, 0, 0, 1), 10)
