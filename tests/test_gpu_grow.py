"""The session table grows instead of filling up (the reference's DashMap, src/packets.rs:330, is
unbounded): before an update call the context doubles the table on the device (k_flow_grow) when
the occupancy reported by the completed updates, projected over the ones in flight, would fill a
partition.  Checked against the C oracle: the table row for row (positions, history state, session
flags), no error bits, the history strings across a growth, and a stream of more than 2^22 = the
previous fixed capacity of distinct flows through the pipelined call."""
import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle

pytestmark = pytest.mark.gpu


def _key_order(a):
    """Row order of flow records by the derived Ord of Session (the oracle's export order)."""
    w = np.ascontiguousarray(a).view(np.uint8).reshape(len(a), N.FLOW_REC_DTYPE.itemsize)[:, :40].copy().view(np.uint32).reshape(len(a), 10)
    ports, pf = w[:, 8], w[:, 9]
    return np.lexsort([ports >> 16, w[:, 7], w[:, 6], w[:, 5], w[:, 4], ports & 0xFFFF, w[:, 3], w[:, 2], w[:, 1],
                       w[:, 0], (pf >> 8) & 0xFF, pf & 0xFF])


def _same_table(g, r):
    assert len(g) == len(r), (len(g), len(r))
    g = g[_key_order(g)].copy()
    g["slot"] = 0
    r = r.copy()
    r["slot"] = 0
    bad = np.flatnonzero((g.view(np.uint8).reshape(len(g), N.FLOW_REC_DTYPE.itemsize) != r.view(np.uint8).reshape(len(r), N.FLOW_REC_DTYPE.itemsize)).any(axis=1))
    assert g.tobytes() == r.tobytes(), "first differing rows: %s" % bad[:5]


def _mk(k):
    return fg.tcp_frame("10.%d.%d.%d" % ((k >> 16) & 255, (k >> 8) & 255, k & 255), 40000 + (k % 7), "8.8.8.8", 443,
                        (fg.SYN, fg.ACK, fg.PSH | fg.ACK, fg.FIN | fg.ACK)[k % 4], 10 + k % 5)


def test_grow_instead_of_table_full():
    """The fixed-table scenario of test_flow_table_small_capacity_and_full (one 512-slot partition,
    then 600 distinct flows) with growth on: the second batch grows the table and nothing is lost."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=512, track_history=True)
    try:
        ref = coracle.Flows()
        batches = [fg.pack([_mk(k) for k in range(300)] * 3)] + \
                  [fg.pack([_mk(k) for k in range(m)]) for m in (600, 1000, 1500, 2000)]
        for frames, offs in batches:
            g = cap.process_frames(frames, offs)
            st = np.zeros(1, dtype=N.STATS_DTYPE)
            ref.update(g.records, st)
            assert g.stats["error"] == 0
            assert g.stats["new_sessions"] == int(st[0]["new_sessions"])
        info = cap.table_info()
        assert info["generation"] >= 2 and info["capacity"] >= 4096, info
        _same_table(cap.export_flows(), ref.export_sorted())
        # history strings follow the flows to their new slots (fb_flow_slot_remap)
        flows = cap.export_flows()
        for r in flows[:: max(1, len(flows) // 50)]:
            h, _ = ref.history(r)
            assert cap.histories.get(int(r["slot"]), "") == h
    finally:
        cap.close()


def test_grow_keeps_the_table_between_synchronous_batches():
    """C4-mix batches with a flow pool four times the initial capacity through fb_process_seg_dev:
    several growths, the table and the batch stats equal the oracle's."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    try:
        ref = coracle.Flows()
        for b in range(5):
            frames, offs = synth.generate(4, 100000, first=b * 100000, n_flows=1 << 19)
            g = cap.process_frames_seg(frames, offs)
            r_out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
            st = np.zeros(1, dtype=N.STATS_DTYPE)
            ref.update(r_out, st)
            assert g.stats["error"] == 0
            assert g.stats["new_sessions"] == int(st[0]["new_sessions"])
            assert g.stats["updated_sessions"] == int(st[0]["updated_sessions"])
        assert cap.table_info()["generation"] >= 1
        _same_table(cap.export_flows(), ref.export_sorted())
    finally:
        cap.close()


def test_stream_more_than_4m_flows_async():
    """> 2^22 distinct flows (the old fixed capacity) streamed through fb_process_seg_async_dev from
    a 2^21-slot start: the table grows past 2^22 slots and stays row-equal to the oracle, with no
    error bits in any batch's stats.  The host joins each batch (as a capture loop reading its
    stats does), so each growth decision sees the previous batch's report."""
    n, batches = 1 << 20, 9
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 21, max_batch_packets=n)
    stream = N.Stream()
    keep = []
    ref = coracle.Flows()
    cfg = coracle.make_cfg(2)
    stats = []
    try:
        nseg = (n + 63) // 64
        sets = [[None, None, N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4),
                 N.DeviceBuffer(N.STATS_DTYPE.itemsize)] for _ in range(2)]
        for b in range(batches):
            frames, offs = synth.generate(2, n, first=b * n, n_flows=1 << 23)
            r_out, _, _, _ = coracle.parse_classify(cfg, frames, offs)
            ref.update(r_out)
            bs = sets[b & 1]
            for x in bs[:2]:
                if x is not None:
                    keep.append(x)
            bs[0] = N.DeviceBuffer(frames.nbytes).upload(frames)
            bs[1] = N.DeviceBuffer(offs.nbytes).upload(offs)
            N.check(lib.fb_process_seg_async_dev(cap.ctx, bs[0].ptr, frames.nbytes, bs[1].ptr, n, bs[2].ptr,
                                                 bs[3].ptr, None, bs[4].ptr, stream.ptr))
            N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
            stream.sync()
            stats.append(bs[4].download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)[0].copy())
        assert all(int(s["error"]) == 0 for s in stats), [int(s["error"]) for s in stats]
        assert sum(int(s["new_sessions"]) for s in stats) == ref.count()
        info = cap.table_info()
        assert ref.count() > (1 << 22) and info["capacity"] > (1 << 22), (ref.count(), info)
        _same_table(cap.export_flows(), ref.export_sorted())
    finally:
        for bs in sets:
            for x in bs:
                if x is not None:
                    x.free()
        for x in keep:
            x.free()
        cap.close()


def test_stream_async_without_joins_grows_in_time():
    """The C4 bench's calling pattern with growth on: fb_process_seg_async_dev batches enqueued back
    to back with two rotating buffer sets and NO join or host read between them (the host runs
    ahead of the device), past the initial capacity and across several growths.  Each growth
    decision reads the report of the update two calls back (maybe_grow waits for it), so no batch
    may report error bit 4 (FB_ERR_TABLE_FULL: dropped packets, where the reference's map is
    unbounded), and the table equals the oracle's."""
    n, batches = 1 << 19, 8
    lib = N.gpu_lib()
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 20, max_batch_packets=n)
    stream = N.Stream()
    ref = coracle.Flows()
    cfg = coracle.make_cfg(2)
    bufs, st_bufs = [], []
    try:
        nseg = (n + 63) // 64
        sets = [(N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4)) for _ in range(2)]
        for b in range(batches):  # every batch resident first: the timed loop below only enqueues
            frames, offs = synth.generate(2, n, first=b * n, n_flows=1 << 23)
            r_out, _, _, _ = coracle.parse_classify(cfg, frames, offs)
            ref.update(r_out)
            bufs.append((N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
                         frames.nbytes))
            st_bufs.append(N.DeviceBuffer(N.STATS_DTYPE.itemsize))
        gen0 = cap.table_info()["generation"]
        for b, (d_fr, d_off, nbytes) in enumerate(bufs):
            d_out, d_seg = sets[b & 1]
            N.check(lib.fb_process_seg_async_dev(cap.ctx, d_fr.ptr, nbytes, d_off.ptr, n, d_out.ptr, d_seg.ptr, None,
                                                 st_bufs[b].ptr, stream.ptr))
        N.check(lib.fb_flow_join(cap.ctx, stream.ptr))
        stream.sync()
        stats = [x.download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)[0].copy() for x in st_bufs]
        assert all(int(s["error"]) == 0 for s in stats), [int(s["error"]) for s in stats]
        assert sum(int(s["new_sessions"]) for s in stats) == ref.count()
        assert sum(int(s["new_sessions"]) + int(s["updated_sessions"]) for s in stats) == n * batches - \
            sum(int(s["n_dns"]) for s in stats)
        info = cap.table_info()
        assert info["generation"] >= gen0 + 2 and ref.count() > (1 << 21), (info, ref.count())
        _same_table(cap.export_flows(), ref.export_sorted())
    finally:
        for d_out, d_seg in sets:
            d_out.free()
            d_seg.free()
        for d_fr, d_off, _ in bufs:
            d_fr.free()
            d_off.free()
        for x in st_bufs:
            x.free()
        cap.close()
