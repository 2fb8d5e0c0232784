"""Timed contexts (FB_CFG_TIMED, flodbadd_amd/csrc/fb_time.hip) against the oracle: per-frame capture
timestamps drive the reference's clock-dependent session state -- start_time / last_activity /
end_time, the 5-s segment timeout, current_segment_start / last_segment_end and the interarrival
sum (src/packets.rs:137-200, 352-426) -- compared field by field with the C restatement
(orc_flows_update_timed), itself pinned by the timed KATs (tests/golden/reference_kats.json) and the
independent Python restatement (tests/test_oracle_kat.py).  Covered: the reference's timed KATs on
the GPU, the dense, segmented and pipelined (table-only: update entries) update paths over several
calls, Zipf-hot flows (long per-flow runs), timestamps that go backwards (the negative-interarrival
skip), table growth mid-stream, a full-size C4 batch, and the API's refusals."""
import ctypes as C

import numpy as np
import pytest

import kat
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture, own_ip_table
from flodbadd_amd.sessions import SessionFilter, packets_to_parsed
from oracle import coracle

pytestmark = pytest.mark.gpu

BASE_NS = 1_700_000_000 * 10 ** 9


def frame_times(n, seed, call=0, back=False, gap_ns=1_000_000, jump_p=0.0005):
    """Capture timestamps of a batch: uniform 0..2*gap_ns apart, a fraction jump_p of the frames after a
    0-12 s pause (so a flow's consecutive packets are both closer and farther than the 5-s timeout),
    each call 40 s after the last; back=True: 2 % of the frames step back up to 2 s (non-monotonic
    capture across interfaces)."""
    rng = np.random.default_rng(seed)
    steps = rng.integers(0, 2 * gap_ns, size=n, dtype=np.int64)
    jump = rng.random(n) < jump_p
    steps[jump] += rng.integers(0, 12_000_000_000, size=int(jump.sum()), dtype=np.int64)
    t = BASE_NS + call * 40_000_000_000 + np.cumsum(steps)
    if back:
        b = rng.random(n) < 0.02
        t[b] -= rng.integers(0, 2_000_000_000, size=int(b.sum()), dtype=np.int64)
    return t.astype(np.uint64)


def _gpu_sorted(cap):
    """The GPU table in the oracle's export order (derived Ord) and each flow's time record (joined by
    slot, slot field zeroed)."""
    from flodbadd_amd.distributed import sort_by_ord
    recs, times = cap.export_flows(), cap.export_times()
    assert len(times) == len(recs)
    recs = sort_by_ord(recs)
    tsl = times[np.argsort(times["slot"], kind="stable")]
    idx = np.searchsorted(tsl["slot"], recs["slot"])
    tg = tsl[np.minimum(idx, max(len(tsl) - 1, 0))].copy()
    assert (tg["slot"] == recs["slot"]).all()
    tg["slot"] = 0
    return recs, tg


def _check(cap, ref, tag=""):
    gr, gt = _gpu_sorted(cap)
    er, et = ref.export_sorted(), ref.export_times()
    assert len(gr) == len(er), (tag, len(gr), len(er))
    kb = lambda a: np.ascontiguousarray(a).view(np.uint8).reshape(len(a), -1)[:, :40]  # noqa: E731
    assert (kb(gr) == kb(er)).all(), tag
    bad = np.flatnonzero((gt.view(np.uint8).reshape(len(gt), 64) != et.view(np.uint8).reshape(len(et), 64)).any(axis=1)
                         | (gr["segment_count"] != er["segment_count"]) | (gr["in_segment"] != er["in_segment"]))
    assert bad.size == 0, (tag, bad.size, gt[bad[:3]], et[bad[:3]])
    return len(er)


@pytest.mark.parametrize("case", [c for c in kat.load()["cases"] if c.get("timed")],
                         ids=[c["name"] for c in kat.load()["cases"] if c.get("timed")])
def test_timed_reference_kats_on_gpu(case):
    cap = FlodbaddGpuCapture(0, session_filter=kat.filter_of(case), flow_capacity=1 << 12,
                             own_ips=case["own_ips"], timed=True)
    try:
        pk = kat.packets_of(case)
        res = cap.process_parsed(pk, ts=kat.times_of(case))
        kat.check_case(case, res.records, cap.export_flows(), times=cap.export_times())
        # and field for field the oracle's
        cfg = coracle.make_cfg(int(kat.filter_of(case)), own_ips=own_ip_table(case["own_ips"]))
        recs, _, _ = coracle.process_parsed(cfg, packets_to_parsed(pk))
        ref = coracle.Flows()
        ref.update(recs, ts=kat.times_of(case))
        _check(cap, ref, case["name"])
    finally:
        cap.close()


@pytest.mark.parametrize("path", ["dense", "seg", "async"])
@pytest.mark.parametrize("zipf", [False, True])
def test_timed_multi_call_vs_oracle(path, zipf):
    """Four update calls of a C4-mix stream (3,000-flow pool; Zipf(1.1): a few flows hold thousands of
    packets per batch) through one update path; after each call every flow's time record and timed
    segment state equal the oracle's."""
    kw = dict(n_flows=3000) if not zipf else dict(n_flows=3000, zipf=1, zipf_s=1.1)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 14, timed=True)
    ref = coracle.Flows()
    lib = N.gpu_lib()
    try:
        if path == "async":
            N.check(lib.fb_set_session_records(cap.ctx, 0))  # table-only: the update reads update entries
        keep = []
        for k in range(4):
            n = 60000 + 7 * k
            fr, of = synth.generate(4, n, first=k * 100000, **kw)
            ts = frame_times(n, seed=k, call=k)
            out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
            ref.update(out, ts=ts)
            if path == "dense":
                cap.process_frames(fr, of, ts=ts)
            elif path == "seg":
                cap.process_frames_seg(fr, of, ts=ts)
            else:  # pipelined: the update runs on the context's stream, joined before the export
                nseg = (n + 63) // 64
                bufs = [N.DeviceBuffer(fr.nbytes).upload(fr), N.DeviceBuffer(of.nbytes).upload(of),
                        N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize),
                        N.DeviceBuffer(ts.nbytes).upload(ts)]
                keep.append(bufs)
                N.check(lib.fb_set_frame_times(cap.ctx, bufs[5].ptr))
                N.check(lib.fb_process_seg_async_dev(cap.ctx, bufs[0].ptr, fr.nbytes, bufs[1].ptr, n, bufs[2].ptr,
                                                     bufs[3].ptr, None, bufs[4].ptr, None))
                if k % 2:
                    N.check(lib.fb_flow_join(cap.ctx, None))
                    N.check(lib.fb_stream_sync(None))
            if path != "async" or k % 2:
                flows = _check(cap, ref, "%s call %d" % (path, k))
        assert flows > 1000
        t = ref.export_times()
        assert (t["segment_count"] > 0).any() and (t["last_segment_end_ns"] != N.FB_SEEN_NONE).any()
        assert (t["total_segment_interarrival_ms"] > 0).any() and (t["end_time_ns"] != N.FB_SEEN_NONE).any()
    finally:
        N.check(lib.fb_flow_join(cap.ctx, None))
        N.check(lib.fb_stream_sync(None))
        cap.close()


def test_timed_backwards_timestamps_and_growth():
    """Timestamps that step back (negative interarrival terms are skipped, src/packets.rs:165-179;
    negative gaps never time out) and a table that grows twice mid-stream (the time records follow
    their flows to the new slots)."""
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 11, timed=True)
    ref = coracle.Flows()
    try:
        g0 = cap.table_info()["generation"]
        for k in range(5):
            n = 20000 + 1000 * k
            fr, of = synth.generate(4, n, first=k * 50000, n_flows=500 * 2 ** k)
            ts = frame_times(n, seed=100 + k, call=k, back=True)
            out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
            ref.update(out, ts=ts)
            cap.process_frames_seg(fr, of, ts=ts) if k % 2 else cap.process_frames(fr, of, ts=ts)
            _check(cap, ref, "call %d" % k)
        assert cap.table_info()["generation"] > g0  # it grew
        t = ref.export_times()
        assert (t["segment_interarrival_div"] > 0).any()
    finally:
        cap.close()


def test_timed_full_size_c4():
    """A full C4 batch (10,485,760 IMIX frames, 2^20-flow pool) and a second one 20 s later through the
    pipelined table-only call: every flow's time record equals the oracle's."""
    n = 10 * (1 << 20)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.GlobalOnly, flow_capacity=1 << 21, timed=True,
                             max_batch_packets=n)
    lib = N.gpu_lib()
    ref = coracle.Flows()
    try:
        N.check(lib.fb_set_session_records(cap.ctx, 0))
        keep = []
        for k in range(2):
            fr, of = synth.generate(4, n, first=k * n)
            # ~2 us apart (a flow's consecutive packets ~2 s apart) + ~1 pause per 1M frames: a mix of gaps
            # under and over the timeout
            ts = frame_times(n, seed=7 + k, call=k, gap_ns=2000, jump_p=1e-6)
            out, _, _, _ = coracle.parse_classify(coracle.make_cfg(1), fr, of)
            ref.update(out, ts=ts)
            nseg = (n + 63) // 64
            bufs = [N.DeviceBuffer(fr.nbytes).upload(fr), N.DeviceBuffer(of.nbytes).upload(of),
                    N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize),
                    N.DeviceBuffer(ts.nbytes).upload(ts)]
            keep.append(bufs)
            N.check(lib.fb_set_frame_times(cap.ctx, bufs[5].ptr))
            N.check(lib.fb_process_seg_async_dev(cap.ctx, bufs[0].ptr, fr.nbytes, bufs[1].ptr, n, bufs[2].ptr,
                                                 bufs[3].ptr, None, bufs[4].ptr, None))
            del fr, of, out
        N.check(lib.fb_flow_join(cap.ctx, None))
        N.check(lib.fb_stream_sync(None))
        st = keep[-1][4].download(np.zeros(1, dtype=N.STATS_DTYPE))
        assert int(st[0]["error"]) == 0
        assert _check(cap, ref, "C4") > 1_000_000
    finally:
        cap.close()


def test_timed_api_refusals():
    lib = N.gpu_lib()
    plain = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 10)
    timed = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 10, timed=True)
    try:
        d = N.DeviceBuffer(64)
        assert lib.fb_set_frame_times(plain.ctx, d.ptr) == N.FB_ERR_INVAL  # not a timed context
        out = np.zeros(4, dtype=N.FLOW_TIME_DTYPE)
        n = C.c_uint64()
        assert lib.fb_flow_export_times(plain.ctx, N.ptr(out), 4, C.byref(n), None) == N.FB_ERR_INVAL
        fr, of = synth.generate(4, 1000)
        with pytest.raises(ValueError):
            timed.process_frames(fr, of)  # no timestamps
        # the library refuses an update without frame times before doing anything
        d_fr, d_of = N.DeviceBuffer(fr.nbytes).upload(fr), N.DeviceBuffer(of.nbytes).upload(of)
        d_out, d_st = N.DeviceBuffer(1000 * 56), N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        assert lib.fb_process_dev(timed.ctx, d_fr.ptr, fr.nbytes, d_of.ptr, 1000, d_out.ptr, None, None, d_st.ptr,
                                  None) == N.FB_ERR_INVAL
        assert timed.flow_count() == 0
        ts = frame_times(1000, seed=1)
        timed.process_frames(fr, of, ts=ts)  # and works with them
        ref = coracle.Flows()
        ref.update(coracle.parse_classify(coracle.make_cfg(2), fr, of)[0], ts=ts)
        _check(timed, ref)
    finally:
        plain.close()
        timed.close()
