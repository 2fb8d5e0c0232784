"""Single-pass dense output (k_parse_dense, behind fb_parse_classify_dev / fb_process_dev for frame
batches): tiles b, b + G, ... per block, decoupled look-back with a compute-it-yourself fallback
for late predecessors, records stored at their batch-wide positions.  Bit-exact against the
oracle's batch-wide compaction across hundreds of back-to-back launches of ragged sizes (the 8-bit
status epoch wrapping), with odd record bases, nothing written past the records, the fallback
forced, and at BASELINE's 1M-frame sizes."""
import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from oracle import coracle

pytestmark = pytest.mark.gpu


def _ctx(flt=2):
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    return FlodbaddGpuCapture(0, session_filter=SessionFilter(flt), flow_capacity=0)


class _Dense:
    """Device buffers for one batch and a checked fb_parse_classify_dev call."""

    def __init__(self, frames, offs, flt=2):
        self.frames, self.offs, self.n = frames, offs, len(offs) - 1
        n = max(self.n, 1)
        self.fr = N.DeviceBuffer(max(frames.nbytes, 1)).upload(frames)
        self.of = N.DeviceBuffer(offs.nbytes).upload(offs)
        self.out, self.dns = N.DeviceBuffer(n * 56 + 64), N.DeviceBuffer(n * 16 + 64)
        self.cls, self.st = N.DeviceBuffer(n), N.DeviceBuffer(128)
        self.ref = coracle.parse_classify(coracle.make_cfg(flt), frames, offs)

    def run(self, cap):
        self.out.memset(0x5A)
        self.dns.memset(0x5A)
        N.check(N.gpu_lib().fb_parse_classify_dev(cap.ctx, self.fr.ptr, self.frames.nbytes, self.of.ptr, self.n,
                                                  self.out.ptr, self.dns.ptr, self.cls.ptr, self.st.ptr, None))

    def check(self):
        r_out, r_dns, r_cls, r_st = self.ref
        n = max(self.n, 1)
        st = self.st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        assert int(st[0]["error"]) == 0
        for k in r_st.dtype.names:
            if k in st.dtype.names and k not in ("reserved",):
                assert int(st[0][k]) == int(r_st[0][k]), k
        out = self.out.download(np.zeros(n * 56 + 64, dtype=np.uint8))
        dns = self.dns.download(np.zeros(n * 16 + 64, dtype=np.uint8))
        ns, nd = len(r_out), len(r_dns)
        assert out[: ns * 56].tobytes() == r_out.tobytes()
        assert (out[ns * 56:] == 0x5A).all(), "bytes past the records were written"
        assert dns[: nd * 16].tobytes() == r_dns.tobytes()
        assert (dns[nd * 16:] == 0x5A).all(), "bytes past the DNS records were written"
        if self.n:
            assert np.array_equal(self.cls.download(np.zeros(self.n, dtype=np.uint8)), r_cls)


def test_dense_many_launches_ragged_sizes():
    """300 launches cycling through sizes around the 1024-frame tile and the grid (partial last
    tiles, fewer tiles than blocks, more tiles than blocks): every launch equals the oracle, so
    the status epoch wraps cleanly."""
    sizes = [1, 63, 64, 65, 1023, 1024, 1025, 4097, 30001, 200000, 777777]
    batches = []
    for k, n in enumerate(sizes):
        frames, offs = synth.generate(3 if k % 2 else 2, n, first=11 * k + 1)
        batches.append(_Dense(frames, offs))
    cap = _ctx()
    try:
        for rep in range(300):
            b = batches[(rep * 7) % len(batches)]
            b.run(cap)
            if rep % 3 == 0 or b.n >= 200000:
                b.check()
    finally:
        cap.close()


def test_dense_odd_bases_and_empty_segments():
    """Segments holding 0, 1, 2 ... 64 session records (odd dense bases as often as even: 56-B
    records at an odd index start 8 B off a 16-B boundary), DNS records between them, and whole
    tiles with nothing to emit."""
    frames_l = []
    for s in range(70):
        k = 0 if s % 9 == 4 else (s * 7) % 64 + 1
        for i in range(64):
            if i < k:
                frames_l.append(fg.tcp_frame("10.0.%d.%d" % (s, i), 40000 + i, "8.8.8.8", 443, fg.ACK, i))
            elif i == k and s % 3 == 0:
                frames_l.append(fg.udp_frame("10.0.9.9", 5353 + s, "8.8.4.4", 53, 16))
            else:
                frames_l.append(fg.eth(0x0806, bytes(46)))  # ARP: parse_packet_pcap -> None
    frames_l += [fg.eth(0x0806, bytes(46))] * 2048  # two tiles of nothing
    frames_l += [fg.tcp_frame("10.9.0.1", 40000, "8.8.8.8", 80, fg.SYN, 0)] * 33
    frames, offs = fg.pack(frames_l)
    cap = _ctx()
    try:
        b = _Dense(frames, offs)
        for _ in range(3):
            b.run(cap)
            b.check()
    finally:
        cap.close()


@pytest.mark.parametrize("cid", [2, 3])
def test_dense_full_size(cid):
    """BASELINE configs[1] / [2] sizes (1,048,576 frames) through the single-pass dense kernel,
    GlobalOnly (the FlodbaddCapture default)."""
    frames, offs = synth.generate(cid, 1 << 20, first=5)
    cap = _ctx(1)
    try:
        b = _Dense(frames, offs, flt=1)
        b.run(cap)
        b.check()
    finally:
        cap.close()


def test_dense_lookback_fallback_forced(monkeypatch):
    """fb_debug_set(FB_DEBUG_DENSE_STEAL_POLLS, 0): every look-back that meets a predecessor's unpublished word at once
    computes that tile's sums itself (the path that keeps the kernel safe when some workgroups are
    not running) and CASes them in -- the outputs stay bit-identical."""
    cap = _ctx()
    N.check(N.gpu_lib().fb_debug_set(cap.ctx, N.FB_DEBUG_DENSE_STEAL_POLLS, 0))
    try:
        for k, n in enumerate((1025, 65536, 300001)):
            frames, offs = synth.generate(3, n, first=91 + k)
            b = _Dense(frames, offs)
            for _ in range(2):
                b.run(cap)
                b.check()
    finally:
        cap.close()


def test_dense_corrupted_tile_offset_drops_instead_of_faulting(monkeypatch):
    """A corrupted look-back offset (FB_DEBUG_DENSE_OFFSET_SKEW: half a batch added to every tile's
    batch-wide offset -- what round 4's no-look-back ablation did by adding the real prefix to a
    fixed one, and faulted with an illegal memory access) must not write outside the caller's
    buffers: the slots whose destination passes the batch's n records are dropped and the batch's
    error word has bit 32; a context without the skew is bit-exact again on the same batch."""
    n = 65536
    frames, offs = synth.generate(3, n, first=7)
    cap = _ctx()
    N.check(N.gpu_lib().fb_debug_set(cap.ctx, N.FB_DEBUG_DENSE_OFFSET_SKEW, n // 2))
    try:
        b = _Dense(frames, offs)
        b.run(cap)
        N.check(N.gpu_lib().fb_stream_sync(None))
        st = b.st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        assert int(st[0]["error"]) & 32
        out = b.out.download(np.zeros(n * 56 + 64, dtype=np.uint8))
        dns = b.dns.download(np.zeros(n * 16 + 64, dtype=np.uint8))
        assert (out[n * 56:] == 0x5A).all() and (dns[n * 16:] == 0x5A).all(), "written past the buffers"
        assert int(st[0]["n_session"]) == len(b.ref[0])  # the counts themselves are right
    finally:
        cap.close()
    cap = _ctx()
    try:
        b.run(cap)
        b.check()
    finally:
        cap.close()
