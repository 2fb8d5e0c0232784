"""GPU parity at BASELINE.json's full sizes, bit-exact against the C oracle (it finishes these
sizes in seconds), plus size-independent properties of the same runs.

* C2 / C3: 1,048,576 frames per batch (configs[1], configs[2]); two distinct full batches through
  ONE `fb_parse_classify_seg_batches_dev` launch with the filter bench.py uses (GlobalOnly, the
  `FlodbaddCapture::new` default, src/capture.rs:108) -- the headline launch, batch for batch.
* C4: 10,485,760 IMIX frames (configs[3]) through `fb_process_seg_dev` (parse + session upsert,
  src/packets.rs:202-537), then a second 2M-frame batch that mostly updates existing flows; the
  exported table equals the oracle's DashMap restatement row for row.
"""
import numpy as np
import pytest

from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle
from test_gpu_segmented import _check, _run_batches

pytestmark = pytest.mark.gpu

FULL = 1 << 20


def _conserved(st, n):
    """Every frame lands in exactly one class (src/packets.rs:603-802 returns Some or None; the
    filter at 321-327 drops the rest)."""
    s = st[0]
    assert int(s["n_session"]) + int(s["n_dns"]) + int(s["n_drop"]) + int(s["n_filtered"]) == n
    assert int(s["total_processed"]) == int(s["ipv4_processed"]) + int(s["ipv6_processed"])
    assert int(s["error"]) == 0 and int(s["bad_offsets"]) == 0


@pytest.mark.parametrize("cid", [2, 3])
def test_full_size_headline_launch(gpu_capture, cid):
    batches = [synth.generate(cid, FULL, first=k * FULL) for k in range(2)]
    flt = SessionFilter.GlobalOnly
    gpu_capture.set_filter(flt)
    try:
        res = _run_batches(gpu_capture, batches)
    finally:
        gpu_capture.set_filter(SessionFilter.All)
    for (frames, offs), r in zip(batches, res):
        _check(gpu_capture, frames, offs, flt=int(flt), res=r)
        _conserved(r[3], FULL)


@pytest.mark.parametrize("cid", [2, 3])
@pytest.mark.parametrize("flt", [SessionFilter.LocalOnly, SessionFilter.GlobalOnly])
def test_full_size_filter_drops(gpu_capture, cid, flt):
    """The headline launch at full size on a LAN-heavy variant of the mix (80 % of the flows with a
    LAN dst as well, synth lan_dst_permille): ~40 % of the SESSION frames are local, so LocalOnly
    drops ~60 % and GlobalOnly ~40 % of them (src/packets.rs:321-327, src/sessions.rs:660-672),
    bit-exact against the oracle batch for batch."""
    batches = [synth.generate(cid, FULL, first=k * FULL, lan_dst_permille=800) for k in range(2)]
    gpu_capture.set_filter(flt)
    try:
        res = _run_batches(gpu_capture, batches)
    finally:
        gpu_capture.set_filter(SessionFilter.All)
    for (frames, offs), r in zip(batches, res):
        _check(gpu_capture, frames, offs, flt=int(flt), res=r)
        _conserved(r[3], FULL)
        s = r[3][0]
        kept = int(s["n_session"]) / (int(s["n_session"]) + int(s["n_filtered"]))
        assert (0.3 < kept < 0.5) if flt == SessionFilter.LocalOnly else (0.5 < kept < 0.7), kept


def _void_sorted(arr):
    """Order-independent view of flow rows (table slot zeroed: placement, not content)."""
    arr = arr.copy()
    arr["slot"] = 0
    return np.sort(np.ascontiguousarray(arr).view("V%d" % arr.dtype.itemsize).ravel())


def test_full_size_c4_session_table(gpu_capture):
    cap = gpu_capture
    cap.clear_all_sessions()
    cfg = coracle.make_cfg(int(SessionFilter.All))
    flows = coracle.Flows()
    n_records = 0
    payload = 0
    for n, first in ((10 * FULL, 0), (2 * FULL, 10 * FULL)):
        frames, offs = synth.generate(4, n, first=first)
        g = cap.process_frames_seg(frames, offs)
        r_out, r_dns, r_cls, r_st = coracle.parse_classify(cfg, frames, offs)
        assert np.array_equal(g.cls, r_cls)
        assert g.records.tobytes() == r_out.tobytes(), "session records differ"
        assert g.dns.tobytes() == r_dns.tobytes(), "dns records differ"
        st = np.zeros(1, dtype=N.STATS_DTYPE)
        flows.update(r_out, st)
        assert g.stats["new_sessions"] == int(st[0]["new_sessions"])
        assert g.stats["updated_sessions"] == int(st[0]["updated_sessions"])
        assert g.stats["new_sessions"] + g.stats["updated_sessions"] == g.stats["n_session"]
        n_records += len(r_out)
        payload += int(r_out["packet_length"].astype(np.int64).sum())
        del frames, offs, g, r_out, r_dns, r_cls
    gflows = cap.export_flows()
    rflows = flows.export_sorted()
    assert len(gflows) == len(rflows) == cap.flow_count()
    # size-independent: every record counted once, every payload byte once
    assert int(gflows["orig_pkts"].sum() + gflows["resp_pkts"].sum()) == n_records
    assert int(gflows["outbound_bytes"].sum() + gflows["inbound_bytes"].sum()) == payload
    assert np.array_equal(_void_sorted(gflows), _void_sorted(rflows))
    cap.clear_all_sessions()
    assert cap.flow_count() == 0


def test_full_size_c4_zipf_session_table(gpu_capture):
    """The bench's skewed line at full size: 10M + 2M IMIX frames under Zipf(1.1) flow popularity,
    so ~19K hot (chunk, partition) groups per batch go through k_flow_combine (combined-entry ids
    from its pool, groups past its key table, the hottest flow at ~12 % of the records) -- every
    flow row, counters and ordered fields, equals the oracle's."""
    cap = gpu_capture
    cap.clear_all_sessions()
    cfg = coracle.make_cfg(int(SessionFilter.All))
    flows = coracle.Flows()
    n_records = 0
    for n, first in ((10 * FULL, 0), (2 * FULL, 10 * FULL)):
        frames, offs = synth.generate(4, n, first=first, zipf=1, zipf_s=1.1)
        g = cap.process_frames_seg(frames, offs)
        r_out = coracle.parse_classify(cfg, frames, offs)[0]
        assert g.records.tobytes() == r_out.tobytes(), "session records differ"
        st = np.zeros(1, dtype=N.STATS_DTYPE)
        flows.update(r_out, st)
        assert g.stats["new_sessions"] == int(st[0]["new_sessions"])
        assert g.stats["updated_sessions"] == int(st[0]["updated_sessions"])
        n_records += len(r_out)
        del frames, offs, g, r_out
    gflows = cap.export_flows()
    rflows = flows.export_sorted()
    assert len(gflows) == len(rflows) == cap.flow_count()
    assert int(gflows["orig_pkts"].sum() + gflows["resp_pkts"].sum()) == n_records
    assert int(max(gflows["orig_pkts"] + gflows["resp_pkts"])) > n_records // 20  # the skew is there
    assert np.array_equal(_void_sorted(gflows), _void_sorted(rflows))
    cap.clear_all_sessions()


def test_full_size_c4_pipelined_table_only_bench_path():
    """bench.py's `extra.c4` timed path exactly (bench.py run_config / c4_line): a context with the
    bench's configuration (GlobalOnly, FB_CFG_FIXED_TABLE at 2^21 slots, 2^24 packets per batch),
    `fb_set_session_records(ctx, 0)` (the table is the only output), two device-resident buffer sets
    of 10,485,760 IMIX frames, and five back-to-back `fb_process_seg_async_dev` calls alternating
    between them with no join in between -- each update overlapping the next call's parse on the
    context's own stream -- then `fb_flow_join` and the export.  The two sets hold DIFFERENT batches
    (the bench rotates one batch), so the table must fold five calls of two batches in call order:
    every row, counters, positions, ordered state and segment state, equals the oracle fed the same
    five batches in order (src/packets.rs:329-343, 105-198), and every call's batch stats are clean."""
    import ctypes as C
    lib = N.gpu_lib()
    cfg = N.FbConfig()
    cfg.abi_version = N.FB_ABI_VERSION
    cfg.filter = N.FB_FILTER_GLOBAL_ONLY
    cfg.max_batch_packets = 1 << 24
    cfg.flow_capacity = 1 << 21
    cfg.flags = N.FB_CFG_FIXED_TABLE
    ctx = lib.fb_create(0, C.byref(cfg))
    assert ctx, lib.fb_last_error()
    ctx = C.c_void_p(ctx)
    n = 10 * FULL
    try:
        stream = N.Stream()
        sets, expect = [], []
        for k in range(2):
            frames, offs = synth.generate(4, n, first=k * n)
            nseg = (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
            sets.append((N.DeviceBuffer(frames.nbytes).upload(frames), frames.nbytes,
                         N.DeviceBuffer(offs.nbytes).upload(offs), N.DeviceBuffer(nseg * N.SEG_BYTES),
                         N.DeviceBuffer(nseg * 4)))
            out, _, _, st = coracle.parse_classify(coracle.make_cfg(int(SessionFilter.GlobalOnly)), frames, offs)
            expect.append((out, st))
            del frames, offs
        N.check(lib.fb_set_session_records(ctx, 0))
        calls = [0, 1, 0, 1, 0]
        stats = [N.DeviceBuffer(N.STATS_DTYPE.itemsize) for _ in calls]
        for i, k in enumerate(calls):
            d_fr, nb, d_off, d_out, d_seg = sets[k]
            N.check(lib.fb_process_seg_async_dev(ctx, d_fr.ptr, nb, d_off.ptr, n, d_out.ptr, d_seg.ptr, None,
                                                 stats[i].ptr, stream.ptr))
        N.check(lib.fb_flow_join(ctx, stream.ptr))
        stream.sync()
        flows = coracle.Flows()
        for i, k in enumerate(calls):
            out, est = expect[k]
            ost = np.zeros(1, dtype=N.STATS_DTYPE)
            flows.update(out, ost)
            g = stats[i].download(np.zeros(1, dtype=N.STATS_DTYPE))
            _conserved(g, n)
            for f in ("total_processed", "tcp_processed", "udp_processed", "ipv4_processed", "ipv6_processed",
                      "n_session", "n_dns", "n_drop", "n_filtered"):
                assert int(g[0][f]) == int(est[0][f]), (i, f)
            assert int(g[0]["new_sessions"]) == int(ost[0]["new_sessions"]), i
            assert int(g[0]["updated_sessions"]) == int(ost[0]["updated_sessions"]), i
        cnt = C.c_uint64(0)
        N.check(lib.fb_flow_count(ctx, C.byref(cnt), None))
        gflows = np.zeros(max(cnt.value, 1), dtype=N.FLOW_REC_DTYPE)
        got = C.c_uint64(0)
        N.check(lib.fb_flow_export(ctx, N.ptr(gflows), cnt.value, C.byref(got), None))
        gflows = gflows[: got.value]
        rflows = flows.export_sorted()
        assert len(gflows) == len(rflows) == cnt.value
        assert int(gflows["segment_count"].sum()) > 0 and int((gflows["in_segment"] == 0).sum()) > 0
        assert np.array_equal(_void_sorted(gflows), _void_sorted(rflows))
    finally:
        lib.fb_destroy(ctx)
