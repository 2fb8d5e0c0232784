"""CPU: the DNS parse restatement (oracle/oracle.c orc_dns_parse = dns-parser 0.8.0 Packet::parse
as restated, parity unpinned: the crate is absent from the reference mount and no reference test
parses DNS) on hand-built messages covering each rule, and the resolver bookkeeping
(flodbadd_amd/dns.py DnsResolver = src/dns.rs:35-99) on the oracle's parses."""
import struct

import numpy as np
import pytest

import dnsgen as G
from flodbadd_amd import _native as N
from flodbadd_amd.dns import DnsResolver
from oracle import coracle

S = {k: i for i, k in enumerate(N.DNS_STATUS)}


def parse(b):
    r, nm, ad = coracle.dns_parse(b)
    return N.DNS_STATUS[int(r["status"])], r, nm, ad


def test_well_formed():
    st, r, nm, _ = parse(G.query(0x1234, "www.example.com"))
    assert st == "ok" and nm == b"www.example.com" and r["id"] == 0x1234
    assert int(r["flags"]) == N.DNS_QUERY | N.DNS_HAS_QUESTION
    st, r, nm, ad = parse(G.response(0x1234, "www.example.com",
                                     [("CNAME", "edge.example.net"), ("A", "93.184.216.34"), ("AAAA", "2606:2800::1")]))
    assert st == "ok" and not int(r["flags"]) & N.DNS_QUERY and r["answers"] == 3
    assert [(int(a["family"]), int(a["addr"][0])) for a in ad] == [(2, 0x5DB8D822), (10, 0x26062800)]
    st, r, nm, _ = parse(G.query(7, "4.3.2.1.in-addr.arpa", qtype=12))
    assert st == "ok" and int(r["flags"]) & N.DNS_REVERSE
    st, r, nm, _ = parse(G.query(8, "ip6.arpa", qtype=12))  # no leading dot: not ".ip6.arpa"
    assert st == "ok" and not int(r["flags"]) & N.DNS_REVERSE
    st, r, nm, _ = parse(G.header(9, False))  # no question at all
    assert st == "ok" and int(r["flags"]) == N.DNS_QUERY


@pytest.mark.parametrize("msg,expect", [
    (b"\x12\x34\x01\x00\x00\x01", "header_too_short"),
    (G.query(1, "example.com")[:-6], "unexpected_eof"),                     # question cut
    (G.query(1, "example.com", qtype=65), "invalid_query_type"),            # HTTPS / SVCB
    (G.header(1, False, qd=1) + G.question("x.com", 1, 5), "invalid_query_class"),
    (G.header(1, True, qd=1, an=1) + G.question("x.com") + G.rr(b"\xc0\x0c", 99, b"abcd"), "invalid_type"),
    (G.header(1, True, qd=1, an=1) + G.question("x.com") + G.rr(b"\xc0\x0c", 1, G.a("1.2.3.4"), cls=9), "invalid_class"),
    (G.header(1, True, qd=1, an=1) + G.question("x.com") + G.rr(b"\xc0\x0c", 1, b"\1\2\3\4\5"), "wrong_rdata_length"),
    (G.header(1, True, qd=1, an=1) + G.question("x.com") + G.rr(b"\xc0\x0c", 16, b"\x05ab"), "wrong_rdata_length"),
    (G.header(1, True, qd=1, an=1) + G.question("x.com") + G.rr(b"\xc0\x0c", 15, b"\0\1"), "wrong_rdata_length"),
    (G.header(1, False, qd=1) + b"\x03a\xffc\x00" + struct.pack("!HH", 1, 1), "label_not_ascii"),
    (G.header(1, False, qd=1) + b"\x41abc\x00" + struct.pack("!HH", 1, 1), "unknown_label_format"),
    (G.header(1, False, qd=1) + b"\xc0\x0c" + struct.pack("!HH", 1, 1), "bad_pointer"),   # points to itself
    (G.header(1, False, qd=1) + b"\xc0\x40" + struct.pack("!HH", 1, 1), "unexpected_eof"),  # beyond the message
    (G.header(1, False, qd=1, ar=2) + G.question("x.com") + G.opt() + G.opt(), "additional_opt"),
])
def test_rejections(msg, expect):
    assert parse(msg)[0] == expect


def test_pointer_rules_and_display():
    # forward pointer on the first jump is allowed (largest_pos starts at the message length)
    m = G.header(1, False, qd=1) + b"\xc0\x12" + struct.pack("!HH", 1, 1) + G.name("fwd.example")
    assert parse(m)[0] == "ok" and parse(m)[2] == b"fwd.example"
    # a label then a pointer to a root byte displays a trailing dot ("a.")
    m = G.header(1, False, qd=1) + b"\x01a\xc0\x14" + struct.pack("!HH", 1, 1) + b"\x00"
    st, r, nm, _ = parse(m)
    assert st == "ok" and nm == b"a."
    # a chain of two backward pointers
    base = G.header(2, True, qd=1, an=1) + G.question("mail.example.org")
    cname = G.rr(b"\xc0\x0c", 5, b"\x03www\xc0\x11")  # www + pointer to "example.org"
    st, r, nm, _ = parse(base + cname)
    assert st == "ok" and nm == b"mail.example.org"


def test_many_answers_truncate_addr_list():
    ans = [("A", "10.0.0.%d" % i) for i in range(N.FB_DNS_MAX_ADDRS + 3)]
    st, r, nm, ad = parse(G.response(3, "many.example", ans))
    assert st == "ok" and len(ad) == N.FB_DNS_MAX_ADDRS and int(r["flags"]) & N.DNS_ADDRS_TRUNCATED


def test_resolver_bookkeeping():
    msgs = [G.query(10, "a.example"), G.query(11, "1.0.0.10.in-addr.arpa", qtype=12),
            G.response(10, "a.example", [("A", "1.1.1.1"), ("AAAA", "2001:db8::1")]),
            G.response(12, "orphan.example", [("A", "2.2.2.2")]),   # no pending query: ignored
            G.query(13, "b.example", qtype=65),                     # HTTPS: rejected by the parser
            G.response(13, "b.example", [("A", "3.3.3.3")])]
    parsed = [coracle.dns_parse(m) for m in msgs]
    recs = np.array([p[0] for p in parsed], dtype=N.DNS_MSG_DTYPE)
    names = np.zeros((len(msgs), N.FB_DNS_MAX_NAME), dtype=np.uint8)
    addrs = np.zeros((len(msgs), N.FB_DNS_MAX_ADDRS), dtype=N.FB_IP_DTYPE)
    for i, (_, nm, ad) in enumerate(parsed):
        names[i, : len(nm)] = np.frombuffer(nm, dtype=np.uint8)
        addrs[i, : len(ad)] = ad
    res = DnsResolver()
    res.process(recs, names, addrs)
    got = {str(k): v for k, v in res.resolutions.items()}
    assert got == {"1.1.1.1": "a.example", "2001:db8::1": "a.example"}
    assert res.pending == {}  # 10 answered, 11 reverse (never stored), 13 unparsable
