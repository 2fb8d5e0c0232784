"""GPU parity of the segmented streaming path (fb_parse_classify_seg_dev / fb_process_seg_dev)
against the CPU oracle, bit-exact: per-segment counts, SESSION records and DNS records (densified
in packet order they must equal the oracle's compacted output), per-frame classes, batch stats,
and the session table built from segments."""
import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle

pytestmark = pytest.mark.gpu


def _expected_seg(r_out, r_dns, n):
    """Per-segment (n_session | n_dns << 16) from the oracle's compacted output."""
    nseg = (n + 63) // 64
    cs = np.bincount(r_out["pkt_index"] // 64, minlength=nseg)[:nseg] if len(r_out) else np.zeros(nseg, int)
    cd = np.bincount(r_dns["pkt_index"] // 64, minlength=nseg)[:nseg] if len(r_dns) else np.zeros(nseg, int)
    return (cs | (cd << 16)).astype(np.uint32)


def _run_seg(cap, frames, offs, flow=False):
    """Raw segmented launch: returns (out bytes, seg words, cls, stats)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint32)
    n = offs.size - 1
    nseg = max((n + 63) // 64, 1)
    lib = N.gpu_lib()
    d_fr = N.DeviceBuffer(max(frames.nbytes, 1))
    if frames.nbytes:
        d_fr.upload(frames)
    d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
    d_out = N.DeviceBuffer(nseg * N.SEG_BYTES)
    d_out.memset(0xA5)  # unwritten slots must stay untouched
    d_seg = N.DeviceBuffer(nseg * 4)
    d_cls = N.DeviceBuffer(max(n, 1))
    d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
    fn = lib.fb_process_seg_dev if flow else lib.fb_parse_classify_seg_dev
    N.check(fn(cap.ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, d_seg.ptr, d_cls.ptr, d_st.ptr, None))
    st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
    raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
    seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))[: (n + 63) // 64]
    cls = d_cls.download(np.zeros(max(n, 1), dtype=np.uint8))[:n]
    return raw, seg, cls, st


def _check(cap, frames, offs, flt=2, res=None, **cfg_kw):
    n = len(offs) - 1
    raw, seg, cls, st = _run_seg(cap, frames, offs) if res is None else res
    r_out, r_dns, r_cls, r_st = coracle.parse_classify(coracle.make_cfg(flt, **cfg_kw), frames, offs)
    assert np.array_equal(cls, r_cls)
    assert np.array_equal(seg, _expected_seg(r_out, r_dns, n))
    g_out, g_dns = N.seg_unpack(raw, seg)
    assert g_out.tobytes() == r_out.tobytes(), "session records differ"
    assert g_dns.tobytes() == r_dns.tobytes(), "dns records differ"
    # bytes of a segment outside its records / DNS tail are never written
    for s, w in enumerate(seg.tolist()):
        cs, cd = w & 0xFFFF, w >> 16
        gap = raw[s * N.SEG_BYTES + cs * 56: (s + 1) * N.SEG_BYTES - 16 * cd]
        assert (gap == 0xA5).all(), "segment %d: bytes written outside its records" % s
    for k in N.STATS_FIELDS:
        if k.startswith("reserved") or k in ("new_sessions", "updated_sessions"):
            continue
        assert int(st[0][k]) == (0 if k == "error" else int(r_st[0][k])), k


@pytest.mark.parametrize("config_id,n", [(2, 5000), (3, 5000), (3, 70001), (4, 200000), (2, 64), (3, 63), (3, 65)])
def test_seg_synthetic_vs_oracle(gpu_capture, config_id, n):
    frames, offs = synth.generate(config_id, n)
    _check(gpu_capture, frames, offs)


@pytest.mark.parametrize("flt", [SessionFilter.All, SessionFilter.GlobalOnly, SessionFilter.LocalOnly])
def test_seg_edge_cases(gpu_capture, flt):
    from flodbadd_amd.capture import lan_v6_table, own_ip_table
    frames, offs = fg.pack([f for _, f in fg.edge_cases()] * 3)
    lan = [("2001:db8:abcd:12::1", 64)]
    own = ["192.168.1.1", "10.0.0.5", "2001:db8::1"]
    gpu_capture.set_filter(flt)
    gpu_capture.set_lan_v6(lan)
    gpu_capture.set_own_ips(own)
    try:
        _check(gpu_capture, frames, offs, int(flt), lan_v6=lan_v6_table(lan), own_ips=own_ip_table(own))
    finally:
        gpu_capture.set_filter(SessionFilter.All)
        gpu_capture.set_lan_v6([])
        gpu_capture.set_own_ips([])


def test_seg_tiny_and_dns_heavy(gpu_capture):
    one = [fg.tcp_frame("1.2.3.4", 1000, "5.6.7.8", 80, fg.SYN, 0)]
    buf, offs = fg.pack(one)
    _check(gpu_capture, buf, offs)
    # a segment that is all DNS, one that is mixed, one that is all SESSION
    dns = [fg.udp_frame("10.0.0.2", 5000 + i, "8.8.8.8", 53, 30) for i in range(64)]
    mix = [fg.udp_frame("10.0.0.2", 6000 + i, "8.8.8.8", 53 if i % 3 == 0 else 443, 20) for i in range(64)]
    ses = [fg.tcp_frame("10.0.0.3", 7000 + i, "1.1.1.1", 443, fg.ACK, 10) for i in range(64)]
    buf, offs = fg.pack(dns + mix + ses + dns[:5])
    _check(gpu_capture, buf, offs)


def test_seg_repeated_launches_identical(gpu_capture):
    """300 back-to-back launches (across the 8-bit epoch wrap and both ticket parities) give the
    same segments and stats."""
    frames, offs = synth.generate(3, 30000)
    raw0, seg0, _, st0 = _run_seg(gpu_capture, frames, offs)
    for _ in range(300 // 50):
        for _ in range(49):
            _run_seg(gpu_capture, frames, offs)
        raw, seg, _, st = _run_seg(gpu_capture, frames, offs)
        assert np.array_equal(seg, seg0)
        assert N.seg_unpack(raw, seg)[0].tobytes() == N.seg_unpack(raw0, seg0)[0].tobytes()
        assert st.tobytes() == st0.tobytes()


def test_seg_flow_table_vs_dense(gpu_capture):
    """fb_process_seg_dev builds the same session table as the dense path and the oracle."""
    batches = [synth.generate(4, 60000, first=b * 60000) for b in range(2)] + \
              [synth.generate(4, 100000, first=0, zipf=1, zipf_s=1.1)]
    gpu_capture.clear_all_sessions()
    flows = coracle.Flows()
    cfg = coracle.make_cfg(2)
    for frames, offs in batches:
        g = gpu_capture.process_frames_seg(frames, offs)
        r_out, r_dns, _, _ = coracle.parse_classify(cfg, frames, offs)
        assert g.records.tobytes() == r_out.tobytes()
        r_st = np.zeros(1, dtype=N.STATS_DTYPE)
        flows.update(r_out, r_st)
        assert g.stats["new_sessions"] == int(r_st[0]["new_sessions"])
        assert g.stats["updated_sessions"] == int(r_st[0]["updated_sessions"])
    gf = gpu_capture.export_flows()
    rf = flows.export_sorted()
    from test_gpu_parity import rows_sorted
    assert len(gf) == len(rf) and rows_sorted(gf) == rows_sorted(rf)
    gpu_capture.clear_all_sessions()


def test_seg_partition_handoff_is_per_call(gpu_capture):
    """The fused call's parse hands record partitions to its own update only: fused and split
    calls interleaved on different buffers (split: fb_parse_classify_seg_dev, then
    fb_flow_update_seg_dev on a buffer the fused call never saw; an update of the fused call's
    buffer again with the other batch's records in it) still build the oracle's table."""
    lib = N.gpu_lib()
    bs = [synth.generate(4, 50000 + 777 * (2 - b), first=b * 60000) for b in range(3)]  # A holds batch 2 too
    cap = gpu_capture
    cap.clear_all_sessions()
    flows = coracle.Flows()
    cfg = coracle.make_cfg(2)

    def bufs(frames, offs):
        n = len(offs) - 1
        nseg = (n + 63) // 64
        d_fr = N.DeviceBuffer(frames.nbytes).upload(np.ascontiguousarray(frames))
        d_off = N.DeviceBuffer(offs.nbytes).upload(np.ascontiguousarray(offs, dtype=np.uint32))
        return n, d_fr, d_off, N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), \
            N.DeviceBuffer(N.STATS_DTYPE.itemsize)

    A = bufs(*bs[0])
    B = bufs(*bs[1])
    n, d_fr, d_off, d_out, d_seg, d_st = A
    N.check(lib.fb_process_seg_dev(cap.ctx, d_fr.ptr, bs[0][0].nbytes, d_off.ptr, n, d_out.ptr, d_seg.ptr, None,
                                   d_st.ptr, None))
    n, d_fr, d_off, d_out, d_seg, d_st = B
    N.check(lib.fb_parse_classify_seg_dev(cap.ctx, d_fr.ptr, bs[1][0].nbytes, d_off.ptr, n, d_out.ptr, d_seg.ptr,
                                          None, d_st.ptr, None))
    N.check(lib.fb_flow_update_seg_dev(cap.ctx, d_out.ptr, d_seg.ptr, n, d_st.ptr, None))
    # batch 2 parsed into A's output buffer by a plain call, then updated
    n2, d_fr2, d_off2, _, _, _ = bufs(*bs[2])
    n, _, _, d_out, d_seg, d_st = A
    N.check(lib.fb_parse_classify_seg_dev(cap.ctx, d_fr2.ptr, bs[2][0].nbytes, d_off2.ptr, n2, d_out.ptr, d_seg.ptr,
                                          None, d_st.ptr, None))
    N.check(lib.fb_flow_update_seg_dev(cap.ctx, d_out.ptr, d_seg.ptr, n2, d_st.ptr, None))
    for frames, offs in bs:
        flows.update(coracle.parse_classify(cfg, frames, offs)[0], np.zeros(1, dtype=N.STATS_DTYPE))
    gf = cap.export_flows()
    rf = flows.export_sorted()
    from test_gpu_parity import rows_sorted
    assert len(gf) == len(rf) and rows_sorted(gf) == rows_sorted(rf)
    cap.clear_all_sessions()


def test_seg_parsed_path(gpu_capture):
    """fb_process_parsed_seg_dev == fb_process_parsed_dev on the same SessionPacketData."""
    frames, offs = synth.generate(3, 20000)
    dense = gpu_capture.parse_classify(frames, offs)
    r = dense.records
    parsed = np.zeros(len(r), dtype=N.PARSED_DTYPE)
    for f in ("src_ip", "dst_ip", "src_port", "dst_port", "protocol", "family", "packet_length",
              "ip_packet_length", "tcp_flags", "pkt_index"):
        parsed[f] = r[f]
    parsed["has_flags"] = r["meta"] & N.META_HAS_FLAGS
    n = len(parsed)
    nseg = (n + 63) // 64
    lib = N.gpu_lib()
    d_in = N.DeviceBuffer(parsed.nbytes).upload(parsed)
    d_out = N.DeviceBuffer(nseg * N.SEG_BYTES)
    d_seg = N.DeviceBuffer(nseg * 4)
    d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
    N.check(lib.fb_process_parsed_seg_dev(gpu_capture.ctx, d_in.ptr, n, d_out.ptr, d_seg.ptr, None, d_st.ptr, None))
    seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))
    raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
    g_out, _ = N.seg_unpack(raw, seg)
    d_out2 = N.DeviceBuffer(max(n, 1) * 56)
    d_st2 = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
    N.check(lib.fb_process_parsed_dev(gpu_capture.ctx, d_in.ptr, n, d_out2.ptr, None, d_st2.ptr, None))
    st2 = d_st2.download(np.zeros(1, dtype=N.STATS_DTYPE))
    dense2 = d_out2.download(np.zeros(int(st2[0]["n_session"]), dtype=N.PKT_OUT_DTYPE))
    assert g_out.tobytes() == dense2.tobytes()


def _run_batches(cap, batches):
    """fb_parse_classify_seg_batches_dev over several batches in one launch."""
    lib = N.gpu_lib()
    desc = np.zeros(len(batches), dtype=N.SEG_BATCH_DTYPE)
    keep, outs = [], []
    for k, (frames, offs) in enumerate(batches):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        n = offs.size - 1
        nseg = max((n + 63) // 64, 1)
        d_fr = N.DeviceBuffer(max(frames.nbytes, 1))
        if frames.nbytes:
            d_fr.upload(frames)
        d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
        d_out = N.DeviceBuffer(nseg * N.SEG_BYTES)
        d_out.memset(0xA5)
        d_seg, d_cls, d_st = N.DeviceBuffer(nseg * 4), N.DeviceBuffer(max(n, 1)), N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        d_st.memset(0x5A)  # every batch's stats must be written, empty ones included
        desc[k] = (d_fr.ptr.value, frames.nbytes, d_off.ptr.value, n, 0, d_out.ptr.value, d_seg.ptr.value,
                   d_cls.ptr.value, d_st.ptr.value)
        keep += [d_fr, d_off]
        outs.append((n, nseg, d_out, d_seg, d_cls, d_st))
    N.check(lib.fb_parse_classify_seg_batches_dev(cap.ctx, N.ptr(desc), len(batches), None))
    res = []
    for n, nseg, d_out, d_seg, d_cls, d_st in outs:
        st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
        seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))[: (n + 63) // 64]
        cls = d_cls.download(np.zeros(max(n, 1), dtype=np.uint8))[:n]
        res.append((raw, seg, cls, st))
    return res


def test_seg_batches_one_launch(gpu_capture):
    """Several batches of different shapes (an empty one, a 1-frame one, IMIX, edge frames) in
    one launch: each batch equals the oracle exactly as a separate launch would."""
    batches = [synth.generate(2, 5000), fg.pack([]), synth.generate(3, 70001),
               fg.pack([fg.tcp_frame("1.2.3.4", 1000, "5.6.7.8", 80, fg.SYN, 0)]),
               fg.pack([f for _, f in fg.edge_cases()] * 3), synth.generate(4, 200000, first=7)]
    for rep in range(3):  # across the per-batch stats words' reuse
        for (frames, offs), res in zip(batches, _run_batches(gpu_capture, batches)):
            _check(gpu_capture, frames, offs, res=res)
    full = [synth.generate(2, 1 << 16, first=k << 16) for k in range(N.FB_MAX_SEG_BATCHES)]
    for (frames, offs), res in zip(full, _run_batches(gpu_capture, full)):
        _check(gpu_capture, frames, offs, res=res)


def test_seg_batches_rejects_bad_counts(gpu_capture):
    lib = N.gpu_lib()
    desc = np.zeros(N.FB_MAX_SEG_BATCHES + 1, dtype=N.SEG_BATCH_DTYPE)
    assert lib.fb_parse_classify_seg_batches_dev(gpu_capture.ctx, N.ptr(desc), 0, None) == N.FB_ERR_INVAL
    assert lib.fb_parse_classify_seg_batches_dev(gpu_capture.ctx, N.ptr(desc), len(desc), None) == N.FB_ERR_INVAL
    assert lib.fb_parse_classify_seg_batches_dev(gpu_capture.ctx, N.ptr(desc), 1, None) == N.FB_ERR_INVAL  # no stats
