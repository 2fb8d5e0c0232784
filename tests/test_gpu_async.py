"""fb_process_seg_async_dev (the pipelined fused call: each batch's table update on the context's
own stream, overlapping the next batch's parse) gives the same table, the same per-batch stats and
the same last-update history as fb_process_seg_dev over the same batches -- with two rotating
buffer sets (overlap), with one buffer set reused every batch (the call waits for the previous
update), mixed with synchronous calls, and with table reads issued without an explicit join."""
import ctypes as C

import numpy as np
import pytest

from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture
from flodbadd_amd.sessions import SessionFilter
from test_gpu_parity import rows_sorted

pytestmark = pytest.mark.gpu


def _batches():
    b = [synth.generate(4, 60000, first=k * 60000, zipf=1, zipf_s=1.1) for k in range(4)]
    b.append(synth.generate(4, 90000, first=400000))  # uniform flows, a larger batch
    return b


def _keyed_history(cap, n_slots, flows):
    """{40-B key: the last update's characters} (slots are placement, so keyed by the flow key)."""
    by_slot = {int(r["slot"]): r.tobytes()[:40] for r in flows}
    return {by_slot[s]: h for s, h in cap.flow_history(n_slots).items()}


def _run(batches, modes, n_sets):
    """Process `batches` with modes[i] in {"sync", "async"}; buffer set i % n_sets per batch."""
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    stream = N.Stream()
    keep = []
    try:
        nmax = max(len(o) - 1 for _, o in batches)
        nseg = (nmax + 63) // 64
        sets = [(N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize))
                for _ in range(n_sets)]
        stats = []
        for i, ((frames, offs), mode) in enumerate(zip(batches, modes)):
            d_fr = N.DeviceBuffer(frames.nbytes).upload(frames)
            d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
            keep += [d_fr, d_off]
            d_out, d_seg, d_st = sets[i % n_sets]
            fn = lib.fb_process_seg_async_dev if mode == "async" else lib.fb_process_seg_dev
            N.check(fn(cap.ctx, d_fr.ptr, frames.nbytes, d_off.ptr, len(offs) - 1, d_out.ptr, d_seg.ptr, None,
                       d_st.ptr, stream.ptr))
            if n_sets >= len(batches) or i == len(batches) - 1:
                stats.append(d_st)
        N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
        stream.sync()
        st = [s.download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr).tobytes() for s in stats]
        flows = cap.export_flows()  # joins the update stream itself (a no-op after the join above)
        n_last = (len(batches[-1][1]) - 1 + 63) // 64 * 64
        hist = _keyed_history(cap, n_last, flows)
        cnt = C.c_uint64()
        N.check(lib.fb_flow_count(cap.ctx, C.byref(cnt), None))
        return rows_sorted(flows), st, hist, int(cnt.value)
    finally:
        for b in keep:
            b.free()
        cap.close()


@pytest.fixture(scope="module")
def reference():
    b = _batches()
    return b, _run(b, ["sync"] * len(b), len(b))


@pytest.mark.parametrize("modes,n_sets", [
    (["async"] * 5, 5),                                 # every batch its own buffers: per-batch stats compared
    (["async"] * 5, 2),                                 # two rotating sets: parse k+1 overlaps update k
    (["async"] * 5, 1),                                 # one set: each call waits for the previous update
    (["async", "async", "sync", "async", "async"], 2),  # a synchronous call in between joins first
], ids=["own-buffers", "two-sets", "one-set", "mixed"])
def test_async_equals_sync(reference, modes, n_sets):
    batches, (ref_rows, ref_stats, ref_hist, ref_cnt) = reference
    rows, st, hist, cnt = _run(batches, modes, n_sets)
    assert cnt == ref_cnt and rows == ref_rows
    assert st == (ref_stats if n_sets >= len(batches) else ref_stats[-1:])
    assert hist == ref_hist


def test_async_table_reads_join(reference):
    """Export / count right after async calls, with no explicit fb_flow_join: the entry points
    join the update stream themselves."""
    batches, (ref_rows, _, _, ref_cnt) = reference
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    keep = []
    try:
        nseg = (max(len(o) - 1 for _, o in batches) + 63) // 64
        for i, (frames, offs) in enumerate(batches):
            bufs = [N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
                    N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize)]
            keep += bufs
            d_fr, d_off, d_out, d_seg, d_st = bufs
            N.check(lib.fb_process_seg_async_dev(cap.ctx, d_fr.ptr, frames.nbytes, d_off.ptr, len(offs) - 1, d_out.ptr,
                                                 d_seg.ptr, None, d_st.ptr, None))
        assert cap.flow_count() == ref_cnt
        assert rows_sorted(cap.export_flows()) == ref_rows
    finally:
        for b in keep:
            b.free()
        cap.close()


def test_async_empty_batch_and_table_full():
    """An empty batch through the pipelined call counts as an update call (as in the synchronous
    one); a batch that overflows a partition reports TABLE_FULL in its stats after the join, and
    the context recovers for the next call."""
    import framegen as fg
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=512, grow=False)
    mk = lambda k: fg.tcp_frame("10.1.%d.%d" % (k >> 8, k & 255), 40000, "8.8.8.8", 443, fg.ACK, 10)
    stream = N.Stream()
    keep = []

    def issue(frames, offs):
        n = len(offs) - 1
        nseg = max((n + 63) // 64, 1)
        b = [N.DeviceBuffer(max(frames.nbytes, 1)), N.DeviceBuffer(offs.nbytes).upload(offs),
             N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize)]
        if frames.nbytes:
            b[0].upload(frames)
        keep.extend(b)
        N.check(lib.fb_process_seg_async_dev(cap.ctx, b[0].ptr, frames.nbytes, b[1].ptr, n, b[2].ptr, b[3].ptr, None,
                                             b[4].ptr, stream.ptr))
        return b[4]

    try:
        issue(*fg.pack([mk(k) for k in range(300)]))
        issue(*fg.pack([]))
        st_full = issue(*fg.pack([mk(k) for k in range(600)]))
        N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
        stream.sync()
        st = st_full.download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)
        assert int(st[0]["error"]) & 4  # partition full
        # the host-side error path resets the launch scratch; the table still answers
        cap.clear_all_sessions()
        g = cap.process_frames(*fg.pack([mk(k) for k in range(200)]))
        assert len(g.records) == 200 and cap.flow_count() == 200
    finally:
        for b in keep:
            b.free()
        cap.close()


def test_table_only_equals_records(reference):
    """fb_set_session_records(ctx, 0) (the reference's capture loop keeps only the table): the same
    table, per-batch stats and history through the pipelined call; no SESSION record is stored in
    d_out, while the segment counts and the DNS side records at the segment tails are."""
    from oracle import coracle
    batches, (ref_rows, ref_stats, ref_hist, ref_cnt) = reference
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    stream = N.Stream()
    keep = []
    try:
        N.check(lib.fb_set_session_records(cap.ctx, 0))
        outs = []
        for frames, offs in batches:
            n = len(offs) - 1
            nseg = (n + 63) // 64
            b = [N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
                 N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize)]
            b[2].memset(0x5A)
            keep += b
            N.check(lib.fb_process_seg_async_dev(cap.ctx, b[0].ptr, frames.nbytes, b[1].ptr, n, b[2].ptr, b[3].ptr,
                                                 None, b[4].ptr, stream.ptr))
            outs.append((frames, offs, nseg, b[2], b[3], b[4]))
        N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
        stream.sync()
        st = [o[5].download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr).tobytes() for o in outs]
        assert st == ref_stats
        flows = cap.export_flows()
        assert cap.flow_count() == ref_cnt and rows_sorted(flows) == ref_rows
        n_last = (len(batches[-1][1]) - 1 + 63) // 64 * 64
        assert _keyed_history(cap, n_last, flows) == ref_hist
        for frames, offs, nseg, d_out, d_seg, _ in outs:
            seg = d_seg.download(np.zeros(nseg, dtype=np.uint32))
            raw = d_out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8)).reshape(nseg, N.SEG_BYTES)
            r_out, r_dns, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
            assert int((seg & 0xFFFF).sum()) == len(r_out) and int((seg >> 16).sum()) == len(r_dns)
            dns = []
            for s in range(nseg):
                cs, cd = int(seg[s] & 0xFFFF), int(seg[s] >> 16)
                assert (raw[s, :cs * 56] == 0x5A).all(), "a SESSION record was stored"
                for j in range(cd):
                    dns.append(raw[s, N.SEG_BYTES - 16 * (j + 1):N.SEG_BYTES - 16 * j].tobytes())
            assert b"".join(dns) == r_dns.tobytes()
    finally:
        N.check(lib.fb_set_session_records(cap.ctx, 1))
        for b in keep:
            b.free()
        cap.close()


@pytest.mark.parametrize("v6_permille", [1000, 500], ids=["v6-only", "v6-half"])
def test_table_only_ipv6_segments(v6_permille):
    """IPv6-heavy batches through the pipelined table-only call: an IPv6 key takes two 32-B update
    units, so an all-IPv6 segment fills its 128-unit region exactly.  The table equals the C
    oracle's row for row, and each batch's new / updated counts equal the oracle's."""
    from oracle import coracle
    from test_gpu_grow import _same_table
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    stream = N.Stream()
    ref = coracle.Flows()
    cfg = coracle.make_cfg(2)
    keep, want, got = [], [], []
    try:
        N.check(lib.fb_set_session_records(cap.ctx, 0))
        for k in range(4):
            frames, offs = synth.generate(4, 70000 + 64 * k + 17, first=k * 80000, v6_permille=v6_permille,
                                          dns_permille=0, n_flows=1 << 15)
            r_out, _, _, _ = coracle.parse_classify(cfg, frames, offs)
            st = np.zeros(1, dtype=N.STATS_DTYPE)
            ref.update(r_out, st)
            want.append((int(st[0]["new_sessions"]), int(st[0]["updated_sessions"])))
            n = len(offs) - 1
            nseg = (n + 63) // 64
            b = [N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
                 N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize)]
            keep += b
            N.check(lib.fb_process_seg_async_dev(cap.ctx, b[0].ptr, frames.nbytes, b[1].ptr, n, b[2].ptr, b[3].ptr,
                                                 None, b[4].ptr, stream.ptr))
            got.append(b[4])
        N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
        stream.sync()
        st = [g.download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)[0] for g in got]
        assert [int(s["error"]) for s in st] == [0] * len(st)
        assert [(int(s["new_sessions"]), int(s["updated_sessions"])) for s in st] == want
        _same_table(cap.export_flows(), ref.export_sorted())
    finally:
        N.check(lib.fb_set_session_records(cap.ctx, 1))
        for b in keep:
            b.free()
        cap.close()
