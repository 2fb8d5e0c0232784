"""Dense output built from the segmented kernel (fb_compact.hip, fb_seg_compact_dev) and the
dense entry points that now run on it (fb_parse_classify_dev, fb_process_parsed_dev,
fb_process_dev): bit-exact against the oracle's batch-wide compaction, with odd record bases
(the 8-B head / tail split of the copy), DNS-only / records-only compaction, nothing written past
the records, and two contexts streaming dense batches concurrently on two streams -- the path has
no inter-workgroup wait, so kernels sharing the device cannot starve it (the look-back kernel this
replaced could time out there)."""
import ctypes as C

import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from oracle import coracle
from test_gpu_segmented import _run_seg

pytestmark = pytest.mark.gpu


def _compact(cap, raw, seg, n, want_out=True, want_dns=True):
    nseg = len(seg)
    d_so = N.DeviceBuffer(max(raw.nbytes, 1)).upload(raw)
    d_sg = N.DeviceBuffer(max(nseg * 4, 4)).upload(np.ascontiguousarray(seg, dtype=np.uint32))
    d_out = N.DeviceBuffer(max(n, 1) * 56 + 64)
    d_dns = N.DeviceBuffer(max(n, 1) * 16 + 64)
    d_out.memset(0x5A)
    d_dns.memset(0x5A)
    N.check(N.gpu_lib().fb_seg_compact_dev(cap.ctx, d_so.ptr, d_sg.ptr, n, d_out.ptr if want_out else None,
                                           d_dns.ptr if want_dns else None, None))
    out = d_out.download(np.zeros(max(n, 1) * 56 + 64, dtype=np.uint8))
    dns = d_dns.download(np.zeros(max(n, 1) * 16 + 64, dtype=np.uint8))
    return out, dns


@pytest.mark.parametrize("config_id,n,first", [(3, 50000, 5), (2, 30001, 9), (3, 777, 1)])
def test_seg_compact_vs_oracle(gpu_capture, config_id, n, first):
    frames, offs = synth.generate(config_id, n, first=first)
    raw, seg, _, st = _run_seg(gpu_capture, frames, offs)
    r_out, r_dns, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    ns, nd = len(r_out), len(r_dns)
    assert int(st[0]["n_session"]) == ns and int(st[0]["n_dns"]) == nd
    for want_out, want_dns in ((True, True), (True, False), (False, True)):
        out, dns = _compact(gpu_capture, raw, seg, n, want_out, want_dns)
        if want_out:
            assert out[: ns * 56].tobytes() == r_out.tobytes()
            assert (out[ns * 56:] == 0x5A).all(), "bytes past the records were written"
        else:
            assert (out == 0x5A).all()
        if want_dns:
            assert dns[: nd * 16].tobytes() == r_dns.tobytes()
            assert (dns[nd * 16:] == 0x5A).all()
        else:
            assert (dns == 0x5A).all()


def test_seg_compact_odd_bases(gpu_capture):
    """Segments holding 1, 2, 3 ... records, so the dense base of a segment is odd as often as even
    (56-B records: an odd base starts 8 B off a 16-B boundary)."""
    frames_l = []
    for s in range(40):
        k = (s * 7) % 64 + 1  # sessions in this segment, the rest dropped (ARP)
        for i in range(64):
            if i < k:
                frames_l.append(fg.tcp_frame("10.0.%d.%d" % (s, i), 40000 + i, "8.8.8.8", 443, fg.ACK, i))
            elif i == k and s % 3 == 0:
                frames_l.append(fg.udp_frame("10.0.9.9", 5353 + s, "8.8.4.4", 53, 16))
            else:
                frames_l.append(fg.eth(0x0806, bytes(46)))  # ARP: parse_packet_pcap -> None
    frames, offs = fg.pack(frames_l)
    n = len(offs) - 1
    raw, seg, _, _ = _run_seg(gpu_capture, frames, offs)
    r_out, r_dns, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    out, dns = _compact(gpu_capture, raw, seg, n)
    assert out[: len(r_out) * 56].tobytes() == r_out.tobytes()
    assert dns[: len(r_dns) * 16].tobytes() == r_dns.tobytes()


def test_seg_compact_empty_and_bad_args(gpu_capture):
    lib = N.gpu_lib()
    assert lib.fb_seg_compact_dev(gpu_capture.ctx, None, None, 0, None, None, None) == N.FB_OK
    assert lib.fb_seg_compact_dev(gpu_capture.ctx, None, None, 10, None, None, None) == N.FB_ERR_INVAL
    assert lib.fb_seg_compact_dev(None, None, None, 0, None, None, None) == N.FB_ERR_INVAL


def test_dense_two_contexts_concurrent():
    """Two contexts, each on its own stream, enqueue dense calls back to back without syncing:
    both streams' kernels share the device, and every batch still equals the oracle."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    lib = N.gpu_lib()
    caps = [FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0) for _ in range(2)]
    streams = []
    try:
        work = []
        for k, cap in enumerate(caps):
            s = C.c_void_p()
            N.check(lib.fb_stream_create(C.byref(s)))
            streams.append(s)
            for j in range(3):
                frames, offs = synth.generate(3, 200000, first=1000 * k + 17 * j)
                n = len(offs) - 1
                bufs = dict(fr=N.DeviceBuffer(frames.nbytes).upload(frames), of=N.DeviceBuffer(offs.nbytes).upload(offs),
                            out=N.DeviceBuffer(n * 56), dns=N.DeviceBuffer(n * 16), st=N.DeviceBuffer(128))
                work.append((cap, s, frames, offs, bufs))
        for rep in range(4):  # interleaved: ctx0 batch, ctx1 batch, ... all in flight together
            for cap, s, frames, offs, b in work:
                N.check(lib.fb_parse_classify_dev(cap.ctx, b["fr"].ptr, frames.nbytes, b["of"].ptr, len(offs) - 1,
                                                  b["out"].ptr, b["dns"].ptr, None, b["st"].ptr, s))
        for s in streams:
            N.check(lib.fb_stream_sync(s))
        for cap, s, frames, offs, b in work:
            r_out, r_dns, _, r_st = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
            st = b["st"].download(np.zeros(1, dtype=N.STATS_DTYPE))
            assert int(st[0]["error"]) == 0
            assert int(st[0]["n_session"]) == len(r_out) and int(st[0]["n_dns"]) == len(r_dns)
            out = b["out"].download(np.zeros(len(r_out), dtype=N.PKT_OUT_DTYPE), len(r_out) * 56)
            dns = b["dns"].download(np.zeros(len(r_dns), dtype=N.DNS_OUT_DTYPE), len(r_dns) * 16)
            assert out.tobytes() == r_out.tobytes() and dns.tobytes() == r_dns.tobytes()
    finally:
        for s in streams:
            lib.fb_stream_destroy(s)
        for cap in caps:
            cap.close()


def test_table_full_then_recovers():
    """A flow-table error is reported by the call that hit it; after fb_flow_clear the same
    context processes the next batches normally (the error words are per launch and reset)."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=512, grow=False)
    try:
        mk = lambda k: fg.tcp_frame("10.1.%d.%d" % (k >> 8, k & 255), 40000, "8.8.8.8", 443, fg.ACK, 10)
        with pytest.raises(N.FbError) as ei:
            cap.process_frames(*fg.pack([mk(k) for k in range(600)]))
        assert ei.value.code == N.FB_ERR_TABLE_FULL
        cap.clear_all_sessions()
        for _ in range(3):
            r = cap.process_frames(*fg.pack([mk(k) for k in range(200)]))
            assert r.stats["error"] == 0
        flows = cap.export_flows()
        assert len(flows) == 200 and int(flows["orig_pkts"].sum()) == 600
    finally:
        cap.close()


@pytest.mark.parametrize("flt", [0, 1, 2])
def test_parsed_paths_every_filter(flt):
    """fb_process_parsed_seg_dev and fb_process_parsed_dev against the oracle under each filter:
    SessionPacketData built from a mixed batch, swapped and unswapped keys at odd and even record
    indices (56-B records are 8-B aligned at odd indices)."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    frames, offs = synth.generate(3, 30000, first=3)
    r_out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    parsed = np.zeros(len(r_out), dtype=N.PARSED_DTYPE)
    sw = (r_out["meta"] & N.META_SWAP) != 0  # back to the raw (as-captured) direction
    for a, b in (("src_ip", "dst_ip"), ("src_port", "dst_port")):
        parsed[a] = np.where(sw[:, None] if r_out[a].ndim > 1 else sw, r_out[b], r_out[a])
        parsed[b] = np.where(sw[:, None] if r_out[a].ndim > 1 else sw, r_out[a], r_out[b])
    for f in ("protocol", "family", "packet_length", "ip_packet_length", "tcp_flags", "pkt_index"):
        parsed[f] = r_out[f]
    parsed["has_flags"] = r_out["meta"] & N.META_HAS_FLAGS
    loc = (np.arange(len(parsed)) % 3 == 0) & (parsed["family"] == 2)  # some flows LAN-to-LAN
    parsed["dst_ip"][loc, 0] = 0x0A000001 + np.arange(int(loc.sum()), dtype=np.uint32)
    parsed["src_ip"][loc, 0] = 0xC0A80001
    n = len(parsed)
    e_out, e_cls, e_st = coracle.process_parsed(coracle.make_cfg(flt), parsed)
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter(flt), flow_capacity=0)
    try:
        nseg = (n + 63) // 64
        d_in = N.DeviceBuffer(parsed.nbytes).upload(parsed)
        d_out, d_seg = N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4)
        d_cls, d_st = N.DeviceBuffer(n), N.DeviceBuffer(128)
        N.check(lib.fb_process_parsed_seg_dev(cap.ctx, d_in.ptr, n, d_out.ptr, d_seg.ptr, d_cls.ptr, d_st.ptr, None))
        seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))
        g_out, _ = N.seg_unpack(d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8)), seg)
        assert g_out.tobytes() == e_out.tobytes()
        assert np.array_equal(d_cls.download(np.zeros(n, dtype=np.uint8)), e_cls)
        d_den = N.DeviceBuffer(n * 56)
        N.check(lib.fb_process_parsed_dev(cap.ctx, d_in.ptr, n, d_den.ptr, d_cls.ptr, d_st.ptr, None))
        st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        assert int(st[0]["n_session"]) == len(e_out)
        den = d_den.download(np.zeros(len(e_out), dtype=N.PKT_OUT_DTYPE), len(e_out) * 56)
        assert den.tobytes() == e_out.tobytes()
        assert np.array_equal(d_cls.download(np.zeros(n, dtype=np.uint8)), e_cls)
    finally:
        cap.close()
