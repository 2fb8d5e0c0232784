"""The resident queue-fed parse (fb_seg_queue_*, k_parse_seg_queue): batches handed one call at a
time to ONE running kernel through a ring in pinned host memory, each batch's segmented outputs,
classes and stats bit-exact against the oracle (the layout fb_parse_classify_seg_dev writes) --
ragged and empty batches, more batches than ring slots, an idle gap between submissions, the
configuration captured at create, and an expired queue reporting an error instead of hanging."""
import time

import numpy as np
import pytest

from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture
from flodbadd_amd.queue import DeviceSegBatch, SegQueue
from flodbadd_amd.sessions import SessionFilter
from test_gpu_segmented import _check

pytestmark = pytest.mark.gpu


class _Batch:
    """A test batch: the host arrays the oracle checks against, beside the package's device buffers."""

    def __init__(self, frames, offs, with_cls=True):
        self.frames = np.ascontiguousarray(frames, dtype=np.uint8)
        self.offs = np.ascontiguousarray(offs, dtype=np.uint32)
        self.n = len(self.offs) - 1
        self.dev = DeviceSegBatch(self.frames, self.offs, with_classes=with_cls)

    def reset(self):
        # bytes outside a segment's records must stay untouched (the fills are host copies: while a
        # queue lives its kernel holds the CUs a fill kernel would wait for; upload() completes before
        # the submit)
        self.dev.fill_outputs()

    def result(self):
        return self.dev.raw()


class _Queue(SegQueue):
    def __init__(self, cap, depth, idle_ms=3000):
        super().__init__(cap, depth=depth, idle_ms=idle_ms)

    def submit(self, b):
        return super().submit(b.dev)


def _verify(b, flt, cfg=None):
    from oracle import coracle
    from test_gpu_segmented import _expected_seg
    raw, seg, cls, st = b.result()
    r_out, r_dns, r_cls, r_st = coracle.parse_classify(cfg or coracle.make_cfg(int(flt)), b.frames, b.offs)
    if cls is None:  # no class output asked for
        cls = r_cls
    # compact diagnostics first (a failing bytes comparison of a 1M-frame batch makes pytest diff for minutes)
    es = _expected_seg(r_out, r_dns, b.n)
    bad = np.flatnonzero(seg != es)
    assert bad.size == 0, ("n=%d: %d segment counts differ, first %d: %x vs %x" %
                           (b.n, bad.size, bad[0], int(seg[bad[0]]), int(es[bad[0]])))
    badc = np.flatnonzero(cls != r_cls)
    assert badc.size == 0, ("n=%d: %d classes differ, first at %d" % (b.n, badc.size, badc[0]))
    g_out, g_dns = N.seg_unpack(raw, seg)
    if g_out.tobytes() != r_out.tobytes():
        d = np.flatnonzero(g_out.view(np.uint8).reshape(-1, 56).any(axis=1) != r_out.view(np.uint8).reshape(-1, 56).any(axis=1)
                           if len(g_out) != len(r_out) else
                           (g_out.view(np.uint8).reshape(-1, 56) != r_out.view(np.uint8).reshape(-1, 56)).any(axis=1))
        raise AssertionError("n=%d: %d of %d records differ, first %s" % (b.n, d.size, len(r_out), d[:5]))
    if cfg is None:
        _check(None, b.frames, b.offs, flt=int(flt), res=(raw, seg, cls, st))
    else:  # (the stats against the same oracle run)
        for k in N.STATS_FIELDS:
            if k.startswith("reserved") or k in ("new_sessions", "updated_sessions", "error"):
                continue
            assert int(st[0][k]) == int(r_st[0][k]), k


@pytest.mark.parametrize("depth", [4, 3, 1])
def test_queue_ragged_batches_more_than_slots(depth):
    """depth 3: four ring slots with at most three batches in flight (the kernel's slot ring is a
    power of two); depth 1: every submission waits for the previous batch."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    sizes = [(3, 65537), (2, 64), (3, 1), (2, 0), (3, 6401), (2, 1 << 20), (3, 63), (3, 300001), (2, 65),
             (3, 12345), (2, 128), (3, 70001)]
    batches = [_Batch(*synth.generate(cid, n, first=7 * k), with_cls=k % 3 != 1) for k, (cid, n) in enumerate(sizes)]
    q = _Queue(cap, depth=depth)
    try:
        for b in batches:
            b.reset()
        tickets = [q.submit(b) for b in batches]  # the later submits wait for slots
        for t in tickets:
            q.wait(t)
        for b in batches:
            _verify(b, SessionFilter.All)
        # the same buffers again, twice round the ring, checked after each wait
        for rnd in range(2):
            for b in batches[:6]:
                b.reset()
                q.wait(q.submit(b))
                _verify(b, SessionFilter.All)
    finally:
        q.close()
        cap.close()


def test_queue_idle_gap_and_captured_configuration():
    """GlobalOnly (the FlodbaddCapture default) captured at create; submissions resume after the
    kernel has drained and waited idle (below its limit)."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.GlobalOnly, flow_capacity=0)
    batches = [_Batch(*synth.generate(3, n, first=3 + k)) for k, n in enumerate((40000, 99999, 1 << 18))]
    q = _Queue(cap, depth=2)
    try:
        for rep in range(3):
            for b in batches:
                b.reset()
            ts = [q.submit(b) for b in batches]
            q.wait(ts[-1])
            for t in ts:
                q.wait(t)
            for b in batches:
                _verify(b, SessionFilter.GlobalOnly)
            time.sleep(0.2)  # every wave drains and waits for the next batch
    finally:
        q.close()
        cap.close()


def test_queue_expired_reports_error():
    """A queue idle past idle_ms stops its kernel; a later submission fails instead of hanging."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    b = _Batch(*synth.generate(2, 4096))
    q = _Queue(cap, depth=2, idle_ms=100)
    try:
        b.reset()
        q.wait(q.submit(b))  # within the limit: fine
        _verify(b, SessionFilter.All)
        time.sleep(1.0)
        with pytest.raises(N.FbError) as e:
            q.wait(q.submit(b))
        assert e.value.code == N.FB_ERR_INTERNAL
    finally:
        q.close()
        cap.close()


def test_queue_submission_limit():
    """The kernel numbers batches in 32 bits, so a queue takes at most FB_QUEUE_MAX_SUBMISSIONS
    batches; the submit past its limit fails with FB_ERR_INVAL (here a lowered limit: the same check)
    instead of wrapping, and the batches before it stay exact."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    b = _Batch(*synth.generate(2, 5000))
    q = _Queue(cap, depth=2)
    try:
        with pytest.raises(N.FbError) as e:
            q.set_limit((1 << 32))  # above FB_QUEUE_MAX_SUBMISSIONS
        assert e.value.code == N.FB_ERR_INVAL
        q.set_limit(3)
        for _ in range(3):
            b.reset()
            q.wait(q.submit(b))
            _verify(b, SessionFilter.All)
        with pytest.raises(N.FbError) as e:
            q.submit(b)
        assert e.value.code == N.FB_ERR_INVAL
        with pytest.raises(N.FbError):
            q.set_limit(2)  # below the batches already submitted
    finally:
        q.close()
        cap.close()


def test_one_queue_per_device():
    """A second queue's blocks could never be resident beside the first's: its create fails (instead
    of a kernel that never starts), and succeeds again once the first is destroyed."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    cap2 = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    lib = N.gpu_lib()
    b = _Batch(*synth.generate(3, 5000, first=11))  # (device buffers before the queue: see its create)
    b2 = _Batch(*synth.generate(2, 3000, first=5))
    q = _Queue(cap, depth=2)
    try:
        assert not lib.fb_seg_queue_create(cap2.ctx, 2, 1000)
        assert b"already runs a queue" in lib.fb_last_error()
        b.reset()
        q.wait(q.submit(b))  # the first queue is unaffected
        _verify(b, SessionFilter.All)
    finally:
        q.close()
    q2 = _Queue(cap2, depth=2)
    try:  # (no device buffer is freed while a queue lives: hipFree waits for the queue's kernel)
        b2.reset()
        q2.wait(q2.submit(b2))
        _verify(b2, SessionFilter.All)
    finally:
        q2.close()
        cap.close()
        cap2.close()


def test_queue_lan_v6_own_ips_captured_at_create():
    """LocalOnly with IPv6 LAN prefixes and own IPs: the edge-case frames and an IMIX batch through the
    queue match the oracle under that configuration, although the context is reset to All with no
    prefixes or own IPs right after the queue is created (the queue keeps what it captured)."""
    import framegen as fg
    from flodbadd_amd.capture import lan_v6_table, own_ip_table
    from oracle import coracle
    lan = [("2001:db8:abcd:12::1", 64)]
    own = ["192.168.1.1", "10.0.0.5", "2001:db8::1"]
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.LocalOnly, flow_capacity=0)
    cap.set_lan_v6(lan)
    cap.set_own_ips(own)
    cfg = coracle.make_cfg(int(SessionFilter.LocalOnly), lan_v6=lan_v6_table(lan), own_ips=own_ip_table(own))
    edge = _Batch(*fg.pack([f for _, f in fg.edge_cases()]))
    imix = _Batch(*synth.generate(3, 70001, first=41))
    cap.parse_classify(edge.frames, edge.offs)  # (the configuration uploaded before the queue captures it)
    q = _Queue(cap, depth=2)
    try:
        cap.set_filter(SessionFilter.All)
        cap.set_lan_v6([])
        cap.set_own_ips([])
        for b in (edge, imix):
            b.reset()
            q.wait(q.submit(b))
            _verify(b, SessionFilter.LocalOnly, cfg=cfg)
    finally:
        q.close()
        cap.close()


def test_queue_large_batch_between_small_ones():
    """An 8M-frame IMIX batch (131,072 segments, chunk counters far past one block's share) between
    small batches in the ring, every one bit-exact."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.GlobalOnly, flow_capacity=0)
    batches = [_Batch(*synth.generate(3, n, first=f)) for n, f in ((4097, 5), (1 << 23, 100), (130, 9))]
    q = _Queue(cap, depth=3)
    try:
        for b in batches:
            b.reset()
        ts = [q.submit(b) for b in batches]
        for t in ts:
            q.wait(t)
        for b in batches:
            _verify(b, SessionFilter.GlobalOnly)
    finally:
        q.close()
        cap.close()


@pytest.mark.timeout(180)
def test_shared_queue_builds_the_session_table():
    """One batch per call WITH the upsert: a queue created shared (FB_QUEUE_SHARED, one workgroup per
    CU) parses C4-mix batches while each completed batch is applied to the context's session table on
    a stream of its own (fb_flow_update_seg_dev, K1 / K2 beside the resident kernel); three rotating
    buffer sets, a set reloaded only after its update completed.  The table equals the oracle's fed
    the same batches in order, row for row, and each update ran while the queue lived (no wait for
    the kernel's idle exit)."""
    import time as _t
    from oracle import coracle
    from test_gpu_parity import rows_sorted
    n_max = 120000
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.GlobalOnly, flow_capacity=1 << 17,
                             max_batch_packets=n_max, grow=False)
    batches = [synth.generate(4, 100000 + 977 * k, first=k * 200000, n_flows=40000) for k in range(9)]
    sets = [DeviceSegBatch(*batches[0], max_frames=n_max, max_bytes=max(b[0].nbytes for b in batches))
            for _ in range(3)]
    lib = N.gpu_lib()
    stream, evs = N.Stream(), [N.Event() for _ in range(3)]
    q = SegQueue(cap, depth=4, idle_ms=4000, shared=True)
    ref = coracle.Flows()
    upd_ms = []
    try:
        for k, (fr, of) in enumerate(batches):
            b = sets[k % 3]
            if k >= 3:
                evs[k % 3].wait_spin()  # its previous batch's update is done
            b.load(fr, of)
            b.fill_outputs()
            t = q.submit(b)
            q.wait(t)
            t0 = _t.perf_counter()
            b.update_table(cap, stream.ptr)
            evs[k % 3].record(stream)
            evs[k % 3].wait_spin()
            upd_ms.append((_t.perf_counter() - t0) * 1e3)
            out, _, _, st = b.result()
            assert int(st[0]["error"]) == 0
            ref.update(coracle.parse_classify(coracle.make_cfg(1), fr, of)[0])
        stream.sync()
    finally:
        q.close()
        for b in sets:
            b.free()
    try:
        assert rows_sorted(cap.export_flows()) == rows_sorted(ref.export_sorted())
        assert max(upd_ms) < 2000, upd_ms  # (an update stuck behind the kernel would wait out idle_ms)
    finally:
        cap.close()
