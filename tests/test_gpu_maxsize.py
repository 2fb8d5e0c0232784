"""Near the per-call limits (include/flodbadd_gpu.h: < 2^27 frames, < 4 GiB of frame bytes): one batch
of 62,914,560 64-B C2 frames -- 4.03 GB of frames, frame offsets up to ~2^31.9, 983,040 segments,
record / segment counts far past 2^24 -- through the segmented headline call and the dense call.
The oracle cannot finish the whole batch in seconds, so three 1M-frame slices (the start, the middle,
the end) are checked bit for bit against it (records and DNS records re-based to the slice's first
packet and byte), and the whole batch through size-independent identities: every frame in one class,
the per-segment counts summing to the stats, the classes counting to the stats, the dense records
equal to the segmented ones at the offsets the segment counts give."""
import numpy as np
import pytest

from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle

pytestmark = pytest.mark.gpu

N_BIG = 60 * (1 << 20)
SLICE = 1 << 20


def test_seg_and_dense_near_max_size():
    frames, offs = synth.generate(2, N_BIG, first=0)
    n = N_BIG
    assert frames.nbytes < (1 << 32) and int(offs[-1]) == frames.nbytes
    flt = SessionFilter.GlobalOnly
    cap = FlodbaddGpuCapture(0, session_filter=flt, flow_capacity=0, max_batch_packets=n)
    lib = N.gpu_lib()
    nseg = (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
    bufs = []
    try:
        d_fr = N.DeviceBuffer(frames.nbytes).upload(frames)
        d_of = N.DeviceBuffer(offs.nbytes).upload(offs)
        d_out, d_seg = N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4)
        d_cls, d_st = N.DeviceBuffer(n), N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        bufs += [d_fr, d_of, d_out, d_seg, d_cls, d_st]
        N.check(lib.fb_parse_classify_seg_dev(cap.ctx, d_fr.ptr, frames.nbytes, d_of.ptr, n, d_out.ptr, d_seg.ptr,
                                              d_cls.ptr, d_st.ptr, None))
        N.check(lib.fb_stream_sync(None))
        st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))[0]
        seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))
        cls = d_cls.download(np.zeros(n, dtype=np.uint8))
        raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
        # whole-batch identities
        assert int(st["error"]) == 0 and int(st["bad_offsets"]) == 0
        assert int(st["n_session"]) + int(st["n_dns"]) + int(st["n_drop"]) + int(st["n_filtered"]) == n
        assert int((seg & 0xFFFF).sum(dtype=np.uint64)) == int(st["n_session"])
        assert int((seg >> 16).sum(dtype=np.uint64)) == int(st["n_dns"])
        counts = np.bincount(cls, minlength=4)
        assert int(counts[N.FB_CLASS_SESSION]) == int(st["n_session"])
        assert int(counts[N.FB_CLASS_DNS]) == int(st["n_dns"])
        assert int(counts[N.FB_CLASS_FILTERED]) == int(st["n_filtered"])
        assert int(counts[N.FB_CLASS_DROP]) == int(st["n_drop"])
        # slices against the oracle
        cfg = coracle.make_cfg(int(flt))
        slices = [0, (n // 2) // 64 * 64, n - SLICE]
        for a in slices:
            o0 = int(offs[a])
            sub_frames = frames[o0: int(offs[a + SLICE])]
            sub_offs = (offs[a: a + SLICE + 1] - np.uint32(o0)).astype(np.uint32)
            r_out, r_dns, r_cls, _ = coracle.parse_classify(cfg, sub_frames, sub_offs)
            r_out = r_out.copy()
            r_dns = r_dns.copy()
            r_out["pkt_index"] += a
            r_dns["pkt_index"] += a
            r_dns["payload_offset"] += o0
            s0, s1 = a // 64, (a + SLICE) // 64
            g_out, g_dns = N.seg_unpack(raw[s0 * N.SEG_BYTES: s1 * N.SEG_BYTES], seg[s0:s1])
            assert g_out.tobytes() == r_out.tobytes(), "slice at %d: records differ" % a
            assert g_dns.tobytes() == r_dns.tobytes(), "slice at %d: DNS records differ" % a
            assert np.array_equal(cls[a: a + SLICE], r_cls), "slice at %d: classes differ" % a
        # the dense call on the same batch: the same records at the offsets the segment counts give
        del raw
        d_dout, d_ddns = N.DeviceBuffer(n * 56 + 64), N.DeviceBuffer(n * 16 + 64)
        d_dst = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        bufs += [d_dout, d_ddns, d_dst]
        N.check(lib.fb_parse_classify_dev(cap.ctx, d_fr.ptr, frames.nbytes, d_of.ptr, n, d_dout.ptr, d_ddns.ptr,
                                          None, d_dst.ptr, None))
        N.check(lib.fb_stream_sync(None))
        dst = d_dst.download(np.zeros(1, dtype=N.STATS_DTYPE))[0]
        for k in ("n_session", "n_dns", "n_drop", "n_filtered", "total_processed", "error"):
            assert int(dst[k]) == int(st[k]), k
        ns, nd = int(st["n_session"]), int(st["n_dns"])
        dense = d_dout.download(np.zeros(ns, dtype=N.PKT_OUT_DTYPE))
        ddns = d_ddns.download(np.zeros(nd, dtype=N.DNS_OUT_DTYPE))
        pre_s = np.concatenate([[0], np.cumsum(seg & 0xFFFF, dtype=np.uint64)])
        pre_d = np.concatenate([[0], np.cumsum(seg >> 16, dtype=np.uint64)])
        assert np.all(np.diff(dense["pkt_index"].astype(np.int64)) > 0), "dense records not in packet order"
        for a in slices:
            s0, s1 = a // 64, (a + SLICE) // 64
            o0 = int(offs[a])
            r_out, r_dns, _, _ = coracle.parse_classify(cfg, frames[o0: int(offs[a + SLICE])],
                                                        (offs[a: a + SLICE + 1] - np.uint32(o0)).astype(np.uint32))
            r_out = r_out.copy()
            r_dns = r_dns.copy()
            r_out["pkt_index"] += a
            r_dns["pkt_index"] += a
            r_dns["payload_offset"] += o0
            assert dense[int(pre_s[s0]): int(pre_s[s1])].tobytes() == r_out.tobytes(), "dense slice at %d" % a
            assert ddns[int(pre_d[s0]): int(pre_d[s1])].tobytes() == r_dns.tobytes(), "dense DNS slice at %d" % a
    finally:
        for b in bufs:
            b.free()
        cap.close()
