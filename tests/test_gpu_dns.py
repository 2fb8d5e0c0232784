"""GPU DNS divert parse (fb_dns_parse_dev) against the oracle's restatement of dns-parser 0.8.0
(parity unpinned: the crate is absent from the reference mount), bit-exact on status, id, flags,
counts, the first question's name and the A / AAAA answers: hand-built messages, thousands of
mutated ones (byte flips, truncations, pointer rewrites), and end to end from frames through
parse_classify's DNS side records into the resolver bookkeeping."""
import random
import struct

import numpy as np
import pytest

import dnsgen as G
import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd.dns import DnsResolver, parse_dns
from oracle import coracle

pytestmark = pytest.mark.gpu


def _corpus(seed, n):
    rnd = random.Random(seed)
    base = [G.query(1, "www.example.com"), G.query(2, "a.b.c.d.e.example.org", qtype=28),
            G.query(3, "4.3.2.1.in-addr.arpa", qtype=12), G.query(4, "svc.example", qtype=65),
            G.response(5, "cdn.example.net", [("CNAME", "edge.example.net"), ("A", "93.184.216.34"),
                                              ("AAAA", "2606:2800:220:1::1"), ("A", "93.184.216.35")]),
            G.response(6, "many.example", [("A", "10.0.%d.%d" % (i // 7, i)) for i in range(12)]),
            G.header(7, True, qd=1, an=1, ns=1, ar=2) + G.question("mx.example") +
            G.rr(b"\xc0\x0c", 15, b"\x00\x0a\x04mail\xc0\x0c") +
            G.rr(b"\xc0\x0c", 6, G.name("ns1.example") + G.name("host.example") + b"\0" * 20) +
            G.opt(rdata=b"\x00\x0a\x00\x08" + b"\x01" * 8) + G.rr(b"\xc0\x0c", 16, b"\x03abc\x02de"),
            G.header(8, True, qd=1, an=1) + G.question("srv.example", 33) +
            G.rr(b"\xc0\x0c", 33, b"\0\1\0\2\0\x35" + G.name("target.example"))]
    out = list(base)
    while len(out) < n:
        m = bytearray(rnd.choice(base))
        op = rnd.random()
        if op < 0.4:
            for _ in range(rnd.randint(1, 3)):
                m[rnd.randrange(len(m))] = rnd.randrange(256)
        elif op < 0.6:
            m = m[: rnd.randrange(len(m) + 1)]
        elif op < 0.8:  # rewrite two bytes into a compression pointer somewhere
            i = rnd.randrange(12, max(13, len(m) - 1))
            m[i: i + 2] = struct.pack("!H", 0xC000 | rnd.randrange(len(m) + 4))
        else:  # counts
            m[4: 12] = struct.pack("!HHHH", *[rnd.randrange(4) for _ in range(4)])
        out.append(bytes(m))
    return out


def _run(msgs):
    buf = b"".join(msgs)
    recs = np.zeros(len(msgs), dtype=N.DNS_OUT_DTYPE)
    o = 0
    for i, m in enumerate(msgs):
        recs[i] = (i, o, len(m), 17, 2, 0)
        o += len(m)
    return parse_dns(np.frombuffer(buf, dtype=np.uint8), recs)


def test_dns_parse_vs_oracle():
    msgs = _corpus(1, 6000)
    g_msgs, g_names, g_addrs = _run(msgs)
    seen = set()
    for i, m in enumerate(msgs):
        r, nm, ad = coracle.dns_parse(m, i)
        assert g_msgs[i].tobytes() == r.tobytes(), (i, m.hex(), g_msgs[i], r)
        assert bytes(g_names[i][: len(nm)]) == nm
        assert g_addrs[i][: len(ad)].tobytes() == ad.tobytes()
        seen.add(int(r["status"]))
    assert len(seen) >= 7  # the mutations reach most rejection rules


def test_dns_long_messages_across_the_stage():
    """Messages longer than the kernel's LDS stage (256 B): answers, names and pointers on both
    sides of the boundary, at every byte alignment of the payload (the stage starts at the dword
    holding the first byte), plus their mutations."""
    long = [G.response(9, "long.example", [("A", "192.0.2.%d" % i) for i in range(30)]),
            G.response(10, "mixed.example", [("AAAA", "2001:db8::%x" % i) for i in range(9)] +
                       [("CNAME", "tail-%d.mixed.example" % i) for i in range(6)] + [("A", "198.51.100.1")]),
            G.header(11, True, qd=1, an=2) + G.question("txt.example", 16) +
            G.rr(b"\xc0\x0c", 16, b"\xff" + b"t" * 255) + G.rr(b"\xc0\x0c", 1, bytes([203, 0, 113, 5]))]
    rnd = random.Random(5)
    msgs = []
    for k in range(1200):
        m = bytearray(long[k % len(long)])
        if k >= len(long) * 4 and rnd.random() < 0.7:
            i = rnd.randrange(len(m))
            m[i] = rnd.randrange(256) if rnd.random() < 0.5 else m[i]
            if rnd.random() < 0.3:
                m = m[: rnd.randrange(200, len(m) + 1)]
        msgs.append(bytes(m))
    assert max(len(m) for m in msgs) > 400
    for pad in range(4):  # a pad message shifts every following payload by pad bytes
        batch = [b"\0" * (12 + pad)] + msgs
        g_msgs, g_names, g_addrs = _run(batch)
        for i, m in enumerate(batch):
            r, nm, ad = coracle.dns_parse(m, i)
            assert g_msgs[i].tobytes() == r.tobytes(), (pad, i, m.hex())
            assert bytes(g_names[i][: len(nm)]) == nm
            assert g_addrs[i][: len(ad)].tobytes() == ad.tobytes()


def test_dns_names_alignment_checked():
    """d_names is written a dword at a time: a misaligned pointer is refused up front."""
    from flodbadd_amd import dns as D
    lib = N.gpu_lib()
    msg = G.query(1, "www.example.com")
    rec = np.zeros(1, dtype=N.DNS_OUT_DTYPE)
    rec[0] = (0, 0, len(msg), 17, 2, 0)
    d_fr = N.DeviceBuffer(len(msg)).upload(np.frombuffer(msg, dtype=np.uint8))
    d_dns = N.DeviceBuffer(rec.nbytes).upload(rec)
    d_msg = N.DeviceBuffer(N.DNS_MSG_DTYPE.itemsize)
    d_names = N.DeviceBuffer(2 * N.FB_DNS_MAX_NAME)
    d_addrs = N.DeviceBuffer(N.FB_DNS_MAX_ADDRS * N.FB_IP_DTYPE.itemsize)
    try:
        rc = lib.fb_dns_parse_dev(D._ctx(), d_fr.ptr, len(msg), d_dns.ptr, 1, None, d_msg.ptr, d_names.ptr.value + 2,
                                  d_addrs.ptr, None)
        assert rc == N.FB_ERR_INVAL and b"aligned" in lib.fb_last_error()
        N.check(lib.fb_dns_parse_dev(D._ctx(), d_fr.ptr, len(msg), d_dns.ptr, 1, None, d_msg.ptr, d_names.ptr.value + 4,
                                     d_addrs.ptr, None))
        m = d_msg.download(np.zeros(1, dtype=N.DNS_MSG_DTYPE))
        nm = d_names.download(np.zeros(2 * N.FB_DNS_MAX_NAME, dtype=np.uint8))
        assert int(m[0]["status"]) == 0 and bytes(nm[4: 4 + int(m[0]["name_len"])]) == b"www.example.com"
    finally:
        for b in (d_fr, d_dns, d_msg, d_names, d_addrs):
            b.free()


def test_dns_end_to_end_from_frames(gpu_capture):
    """UDP and DNS-over-TCP frames -> parse_classify (DNS side records) -> GPU parse -> resolver,
    equal to the resolver run on the oracle's parses of the same payloads."""
    q = G.query(0x42, "video.example.com")
    r = G.response(0x42, "video.example.com", [("A", "198.51.100.7"), ("AAAA", "2001:db8::7")])
    q2 = G.query(0x43, "tcp.example.com")
    r2 = G.response(0x43, "tcp.example.com", [("A", "203.0.113.9")])
    frames = [fg.eth(0x0800, fg.ipv4("10.0.0.2", "8.8.8.8", 17, fg.udp(5353, 53, q))),
              fg.tcp_frame("10.0.0.3", 44000, "1.1.1.1", 443, fg.ACK, 20),
              fg.eth(0x0800, fg.ipv4("8.8.8.8", "10.0.0.2", 17, fg.udp(53, 5353, r))),
              fg.eth(0x0800, fg.ipv4("10.0.0.2", "9.9.9.9", 6, fg.tcp(40000, 53, fg.ACK | fg.PSH,
                                                                      struct.pack("!H", len(q2)) + q2))),
              fg.eth(0x0800, fg.ipv4("9.9.9.9", "10.0.0.2", 6, fg.tcp(53, 40000, fg.ACK | fg.PSH,
                                                                      struct.pack("!H", len(r2)) + r2)))]
    buf, offs = fg.pack(frames)
    res = gpu_capture.parse_classify(buf, offs)
    assert len(res.dns) == 4
    gm, gn, ga = parse_dns(buf, res.dns)
    gres = DnsResolver()
    gres.process(gm, gn, ga)
    ores = DnsResolver()
    parsed = [coracle.dns_parse(bytes(buf[d["payload_offset"]: d["payload_offset"] + d["payload_length"]]),
                                int(d["pkt_index"])) for d in res.dns]
    om = np.array([p[0] for p in parsed], dtype=N.DNS_MSG_DTYPE)
    on = np.zeros((len(parsed), N.FB_DNS_MAX_NAME), dtype=np.uint8)
    oa = np.zeros((len(parsed), N.FB_DNS_MAX_ADDRS), dtype=N.FB_IP_DTYPE)
    for i, (_, nm, ad) in enumerate(parsed):
        on[i, : len(nm)] = np.frombuffer(nm, dtype=np.uint8)
        oa[i, : len(ad)] = ad
    ores.process(om, on, oa)
    assert gm.tobytes() == om.tobytes()
    assert gres.resolutions == ores.resolutions
    assert {str(k): v for k, v in gres.resolutions.items()} == {
        "198.51.100.7": "video.example.com", "2001:db8::7": "video.example.com", "203.0.113.9": "tcp.example.com"}


def test_dns_parse_full_size():
    """The bench's DNS workload at full size (synth.dns_workload: 1,048,576 port-53 payloads,
    queries and compressed responses): the parse of every 8th message (131,072) and of the first
    and last 4,096 equals the oracle's, and the batch holds no rejected message."""
    from flodbadd_amd import synth
    payload, recs = synth.dns_workload(1 << 20)
    g_msgs, g_names, g_addrs = parse_dns(payload, recs)
    assert len(g_msgs) == len(recs) == 1 << 20
    idx = sorted(set(range(0, len(recs), 8)) | set(range(4096)) | set(range(len(recs) - 4096, len(recs))))
    for i in idx:
        o, ln = int(recs[i]["payload_offset"]), int(recs[i]["payload_length"])
        r, nm, ad = coracle.dns_parse(payload[o: o + ln].tobytes(), int(recs[i]["pkt_index"]))
        assert g_msgs[i].tobytes() == r.tobytes(), (i, g_msgs[i], r)
        assert bytes(g_names[i][: len(nm)]) == nm
        assert g_addrs[i][: len(ad)].tobytes() == ad.tobytes()
    assert (g_msgs["status"] == 0).all()
