"""get_sessions' read-time SessionFilter and the session flags stored at insert.

The reference keeps is_local_src/dst and is_self_src/dst in SessionInfo from the moment a session
is inserted (src/packets.rs:429-435), while get_sessions (src/capture.rs:1578-1612) and
filter_sessions (src/sessions.rs:678-692) decide LocalOnly / GlobalOnly per query with
is_local_session! / is_global_session!, i.e. is_lan_ip of the session's addresses under the LAN
configuration of that moment (src/sessions.rs:660-672).  CPU tests cover the host-side helpers;
the GPU tests populate a table under All and query it under every filter, before and after the
IPv6 LAN prefixes change, against the C oracle's table."""
import ipaddress
import json
import os

import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd.sessions import (Session, SessionFilter, SessionInfo, filter_sessions, flows_to_sessions,
                                   is_lan_ip)
from oracle import coracle, pyoracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LAN6 = [("2001:db8:1::", 48)]
OWN = ["10.1.1.1", "2001:db8:1::5"]


def _frames():
    """TCP / UDP frames over local-local, local-global and global-global pairs, v4 and v6 (one
    v6 network that is LAN only through the interface prefix LAN6)."""
    pairs = [("10.1.1.1", "192.168.5.9"), ("10.1.1.1", "8.8.8.8"), ("1.2.3.4", "9.9.9.9"),
             ("172.20.0.7", "172.31.255.1"), ("127.0.0.1", "127.0.0.1"), ("169.254.1.1", "224.0.0.5"),
             ("fe80::1", "fd00::2"), ("2001:db8:1::5", "2001:db8:1::9"), ("2001:db8:1::5", "2606:4700::1"),
             ("2a00::1", "2a00::2"), ("2001:db8:2::1", "2001:db8:1::7")]
    out = []
    for k, (a, b) in enumerate(pairs):
        for j in range(4):
            sp, dp = 40000 + k * 10 + j, (443, 22, 5353, 61000)[j]
            out.append(fg.tcp_frame(a, sp, b, dp, fg.SYN if j % 2 else fg.PSH | fg.ACK, 7 * j))
            out.append(fg.tcp_frame(b, dp, a, sp, fg.SYN | fg.ACK, 3))
            out.append(fg.udp_frame(a, sp + 1, b, dp, 11 + j))
    return fg.pack(out)


def _lan_table(prefixes):
    t = np.zeros(len(prefixes), dtype=N.LAN_V6_DTYPE)
    for i, (ip, pfx) in enumerate(prefixes):
        net = ipaddress.IPv6Network("%s/%d" % (ip, pfx), strict=False)
        v = int(net.network_address)
        t[i]["net"] = [(v >> (96 - 32 * w)) & 0xFFFFFFFF for w in range(4)]
        t[i]["prefix"] = pfx
    return t


def _own_table(ips):
    t = np.zeros(len(ips), dtype=N.FB_IP_DTYPE)
    for i, ip in enumerate(ips):
        a = ipaddress.ip_address(ip)
        if a.version == 4:
            t[i]["addr"] = [int(a), 0, 0, 0]
            t[i]["family"] = 2
        else:
            v = int(a)
            t[i]["addr"] = [(v >> (96 - 32 * w)) & 0xFFFFFFFF for w in range(4)]
            t[i]["family"] = 10
    return t


def _oracle_table(frames, offs, lan6):
    cfg = coracle.make_cfg(2, lan_v6=_lan_table(lan6), own_ips=_own_table(OWN))
    out, _, _, _ = coracle.parse_classify(cfg, frames, offs)
    fl = coracle.Flows()
    fl.update(out)
    return out, fl.export_sorted()


def _rows(a):
    a = a.copy()
    a["slot"] = 0
    b, w = a.tobytes(), a.dtype.itemsize
    return sorted(b[i:i + w] for i in range(0, len(b), w))


def _local_now(rec, lan6):
    """is_local_session! of a flow record under the configuration `lan6` (the Python oracle)."""
    pc = pyoracle.Config(lan_v6=lan6)
    s = Session.from_key(rec)
    return pc.is_lan(s.src_ip) and pc.is_lan(s.dst_ip)


# ---- CPU --------------------------------------------------------------------------------------
def test_is_lan_ip_host_helper_matches_reference_vectors():
    """sessions.is_lan_ip on the reference's own is_lan_ip vectors (src/ip.rs:330-456,
    src/sessions.rs:1439-1456, transcribed in reference_kats.json)."""
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        kats = json.load(f)
    lan = kats["lan"]
    assert len(lan["vectors"]) > 10
    prefixes = [tuple(x) for x in lan["lan_v6_prefixes"]]
    for ip, expect in lan["vectors"]:
        assert is_lan_ip(ip, prefixes) == expect, ip
    # interface prefixes of the LAN cache (src/ip.rs:141-156)
    assert is_lan_ip("2001:db8:1::9", LAN6) and not is_lan_ip("2001:db8:2::9", LAN6)
    assert is_lan_ip("2001:db8::1", [("2001:db8::", 32)]) and not is_lan_ip("2001:db9::1", [("2001:db8::", 32)])


def test_filter_sessions_evaluates_locality_at_query_time():
    """filter_sessions uses is_lan_ip now, not the flags stored at insert."""
    mk = lambda a, b, stored: SessionInfo(Session(6, ipaddress.ip_address(a), 1, ipaddress.ip_address(b), 2),
                                          is_local_src=stored, is_local_dst=stored)
    ss = [mk("10.0.0.1", "10.0.0.2", False), mk("10.0.0.1", "8.8.8.8", True),
          mk("2001:db8:1::1", "2001:db8:1::2", False)]
    assert [s.session.dst_port for s in filter_sessions(ss, SessionFilter.All)] == [2, 2, 2]
    loc = filter_sessions(ss, SessionFilter.LocalOnly)
    assert [str(s.session.src_ip) for s in loc] == ["10.0.0.1"] and str(loc[0].session.dst_ip) == "10.0.0.2"
    assert len(filter_sessions(ss, SessionFilter.GlobalOnly)) == 2
    assert len(filter_sessions(ss, SessionFilter.LocalOnly, LAN6)) == 2
    assert len(filter_sessions(ss, SessionFilter.GlobalOnly, LAN6)) == 1


def test_oracle_stores_session_flags_at_insert():
    """The C oracle's table keeps the inserting record's locality / self bits
    (src/packets.rs:429-435); the Python restatement agrees."""
    frames, offs = _frames()
    out, flows = _oracle_table(frames, offs, LAN6)
    pc = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=2, lan_v6=LAN6, own_ips=OWN)
    tab = pyoracle.SessionTable()
    pyoracle.run_batch(pc, frames, offs, tab)
    assert len(tab.sessions) == len(flows)
    for r in flows:
        s = Session.from_key(r)
        p = tab.sessions[(int(s.protocol), s.src_ip, s.src_port, s.dst_ip, s.dst_port)]
        f = int(r["session_flags"])
        assert bool(f & N.SESSION_LOCAL_SRC) == p["is_local_src"] and bool(f & N.SESSION_LOCAL_DST) == p["is_local_dst"]
        assert bool(f & N.SESSION_SELF_SRC) == p["is_self_src"] and bool(f & N.SESSION_SELF_DST) == p["is_self_dst"]
    infos = flows_to_sessions(flows)
    assert sum(i.is_self_src or i.is_self_dst for i in infos) > 0
    assert sum(i.is_local_src and i.is_local_dst for i in infos) > 0
    assert sum(not (i.is_local_src and i.is_local_dst) for i in infos) > 0


# ---- GPU --------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_get_sessions_read_time_filter_gpu():
    """Populate under All, then get_sessions under LocalOnly / GlobalOnly / All equals the oracle's
    table filtered by is_local_session! (capture.rs:1603-1608); after the LAN prefixes change the
    filter follows the new configuration while session_flags keep their insert-time values."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    frames, offs = _frames()
    _, ref = _oracle_table(frames, offs, LAN6)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 12, lan_v6=LAN6, own_ips=OWN)
    try:
        cap.process_frames(frames, offs)
        allf = cap.export_flows()
        assert _rows(allf) == _rows(ref), "table (with session_flags) differs from the oracle"
        for lan6 in (LAN6, []):
            if not lan6:
                cap.set_lan_v6([])  # the LAN cache changes; stored flags do not
            for flt in (SessionFilter.LocalOnly, SessionFilter.GlobalOnly, SessionFilter.All):
                cap.set_filter(flt)
                got = cap.export_flows(flt)
                if flt == SessionFilter.All:
                    want = ref
                else:
                    keep = np.array([_local_now(r, lan6) == (flt == SessionFilter.LocalOnly) for r in ref], dtype=bool)
                    want = ref[keep]
                assert _rows(got) == _rows(want), (flt, lan6)
                infos = cap.get_sessions()
                assert len(infos) == len(want)
                assert [i.session for i in infos] == sorted((Session.from_key(r) for r in want),
                                                             key=lambda s: s.sort_key())
        # both filters are non-trivial on this batch under the original prefixes
        cap.set_lan_v6(LAN6)
        n_loc = len(cap.export_flows(SessionFilter.LocalOnly))
        n_glob = len(cap.export_flows(SessionFilter.GlobalOnly))
        assert n_loc > 0 and n_glob > 0 and n_loc + n_glob == len(ref)
    finally:
        cap.close()
