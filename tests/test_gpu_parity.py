"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Every comparison is on whole records (all 56 bytes), DNS side records, per-frame classes and
batch statistics.  Sizes: hand-built edge cases, seeded synthetic samples the oracle finishes
in seconds, and BASELINE.json's full sizes through size-independent properties.
"""
import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle

pytestmark = pytest.mark.gpu


def _assert_same(gpu, ref):
    g_out, g_dns, g_cls, g_st = gpu.records, gpu.dns, gpu.cls, gpu.stats
    r_out, r_dns, r_cls, r_st = ref
    assert np.array_equal(g_cls, r_cls), "per-frame class mismatch at %s" % np.nonzero(g_cls != r_cls)[0][:10]
    assert g_out.tobytes() == r_out.tobytes(), "session records differ"
    assert g_dns.tobytes() == r_dns.tobytes(), "dns records differ"
    for k in N.STATS_FIELDS:
        if k.startswith("reserved") or k in ("new_sessions", "updated_sessions", "error"):
            continue
        assert g_st[k] == int(r_st[0][k]), k


@pytest.mark.parametrize("flt", [SessionFilter.All, SessionFilter.GlobalOnly, SessionFilter.LocalOnly])
def test_edge_cases(gpu_capture, flt):
    frames, offs = fg.pack([f for _, f in fg.edge_cases()])
    lan = [("2001:db8:abcd:12::1", 64)]
    own = ["192.168.1.1", "10.0.0.5", "2001:db8::1"]
    gpu_capture.set_filter(flt)
    gpu_capture.set_lan_v6(lan)
    gpu_capture.set_own_ips(own)
    try:
        from flodbadd_amd.capture import lan_v6_table, own_ip_table
        cfg = coracle.make_cfg(int(flt), lan_v6=lan_v6_table(lan), own_ips=own_ip_table(own))
        _assert_same(gpu_capture.parse_classify(frames, offs), coracle.parse_classify(cfg, frames, offs))
    finally:
        gpu_capture.set_filter(SessionFilter.All)
        gpu_capture.set_lan_v6([])
        gpu_capture.set_own_ips([])


@pytest.mark.parametrize("config_id,n", [(2, 5000), (3, 5000), (3, 70001), (4, 200000)])
def test_synthetic_vs_oracle(gpu_capture, config_id, n):
    frames, offs = synth.generate(config_id, n)
    cfg = coracle.make_cfg(2)
    _assert_same(gpu_capture.parse_classify(frames, offs), coracle.parse_classify(cfg, frames, offs))


def test_empty_and_tiny_batches(gpu_capture):
    cfg = coracle.make_cfg(2)
    for frames in ([], [fg.tcp_frame("1.2.3.4", 1000, "5.6.7.8", 80, fg.SYN, 0)], [b""] * 3):
        buf, offs = fg.pack(frames)
        _assert_same(gpu_capture.parse_classify(buf, offs), coracle.parse_classify(cfg, buf, offs))


def test_bad_offsets(gpu_capture):
    buf, offs = fg.pack([fg.tcp_frame("1.2.3.4", 1000, "5.6.7.8", 80, fg.SYN, 0)] * 4)
    offs = offs.copy()
    offs[2] = offs[1] - 1          # decreasing
    offs[4] = offs[4] + 1000       # past the end of the buffer
    cfg = coracle.make_cfg(2)
    g = gpu_capture.parse_classify(buf, offs)
    _assert_same(g, coracle.parse_classify(cfg, buf, offs))
    assert g.stats["bad_offsets"] == 2


def test_flow_table_vs_oracle(gpu_capture):
    gpu_capture.clear_all_sessions()
    flows = coracle.Flows()
    cfg = coracle.make_cfg(2)
    for b in range(3):
        frames, offs = synth.generate(4, 60000, first=b * 60000)
        g = gpu_capture.process_frames(frames, offs)
        r_out, r_dns, r_cls, r_st = coracle.parse_classify(cfg, frames, offs)
        assert g.records.tobytes() == r_out.tobytes()
        r_st = np.zeros(1, dtype=N.STATS_DTYPE)
        flows.update(r_out, r_st)
        assert g.stats["new_sessions"] == int(r_st[0]["new_sessions"])
        assert g.stats["updated_sessions"] == int(r_st[0]["updated_sessions"])
    gflows = gpu_capture.export_flows()
    rflows = flows.export_sorted()
    assert len(gflows) == len(rflows)
    assert rows_sorted(gflows) == rows_sorted(rflows)
    gpu_capture.clear_all_sessions()
    assert gpu_capture.flow_count() == 0


def _flows_vs_oracle(cap, batches):
    cap.clear_all_sessions()
    flows = coracle.Flows()
    for frames, offs in batches:
        g = cap.process_frames(frames, offs)
        r_st = np.zeros(1, dtype=N.STATS_DTYPE)
        flows.update(g.records, r_st)  # records are checked against the oracle elsewhere
        assert g.stats["new_sessions"] == int(r_st[0]["new_sessions"])
        assert g.stats["updated_sessions"] == int(r_st[0]["updated_sessions"])
        assert g.stats["error"] == 0
    gflows = cap.export_flows()
    rflows = flows.export_sorted()
    assert len(gflows) == len(rflows)
    assert rows_sorted(gflows) == rows_sorted(rflows)


def test_flow_table_zipf_many_chunks(gpu_capture):
    """One 600k-record batch (37 bucketing chunks) with Zipf(1.1) flow popularity: hot flows put
    thousands of records into one partition; counters must still be exact."""
    _flows_vs_oracle(gpu_capture, [synth.generate(4, 600000, first=0, zipf=1, zipf_s=1.1),
                                   synth.generate(4, 100000, first=600000, zipf=1, zipf_s=1.1)])


def test_flow_table_single_flow_batch(gpu_capture):
    """Every record of the batch on ONE flow (one partition, one slot, all LDS adds collide)."""
    buf, offs = fg.pack([fg.tcp_frame("10.0.0.1", 40000, "8.8.8.8", 443, fg.ACK, 100)] * 50000 +
                        [fg.tcp_frame("8.8.8.8", 443, "10.0.0.1", 40000, fg.ACK, 7)] * 30000)
    _flows_vs_oracle(gpu_capture, [(buf, offs), (buf, offs)])


def test_flow_table_small_capacity_and_full():
    """flow_capacity 512 = one partition, growth off (FB_CFG_FIXED_TABLE): 300 flows fit; 600
    distinct flows report TABLE_FULL."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=512, grow=False)
    try:
        mk = lambda k: fg.tcp_frame("10.1.%d.%d" % (k >> 8, k & 255), 40000, "8.8.8.8", 443, fg.ACK, 10)
        _flows_vs_oracle(cap, [fg.pack([mk(k) for k in range(300)] * 3)])
        with pytest.raises(N.FbError) as ei:
            cap.process_frames(*fg.pack([mk(k) for k in range(600)]))
        assert ei.value.code == N.FB_ERR_TABLE_FULL
    finally:
        cap.close()


def rows_sorted(arr):
    """Order-independent view of a record array: its rows as sorted byte strings (a flow record's
    table slot is placement, not content: it is zeroed, as in the oracle's export)."""
    if arr.dtype.names and "slot" in arr.dtype.names:
        arr = arr.copy()
        arr["slot"] = 0
    b = arr.tobytes()
    w = arr.dtype.itemsize
    return sorted(b[i:i + w] for i in range(0, len(b), w))


# ---- reference known-answer tests through the GPU parsed-packet path --------------------------
import kat  # noqa: E402
from flodbadd_amd.sessions import packets_to_parsed  # noqa: E402

_KATS = kat.load()


_UNTIMED = [c for c in _KATS["cases"] if not c.get("timed")]  # (timed cases: tests/test_gpu_timed.py)


@pytest.mark.parametrize("case", _UNTIMED, ids=[c["name"] for c in _UNTIMED])
def test_reference_kat_on_gpu(gpu_capture, case):
    """process_parsed_packet KATs (src/packets.rs, tests/metrics_test.rs, src/capture.rs) on the
    GPU: keys, counters, derived f64s, history; records byte-identical to the oracle's."""
    from flodbadd_amd.capture import own_ip_table
    gpu_capture.clear_all_sessions()
    gpu_capture.set_filter(kat.filter_of(case))
    gpu_capture.set_own_ips(case["own_ips"])
    try:
        parsed = packets_to_parsed(kat.packets_of(case))
        g = gpu_capture.process_parsed(parsed)
        flows = gpu_capture.export_flows()
        kat.check_case(case, g.records, flows, gpu_capture.flow_history(len(parsed)))
        cfg = coracle.make_cfg(int(kat.filter_of(case)), own_ips=own_ip_table(case["own_ips"]))
        r_out, r_cls, r_st = coracle.process_parsed(cfg, parsed)
        assert g.records.tobytes() == r_out.tobytes()
        assert np.array_equal(g.cls, r_cls)
        assert g.stats["total_processed"] == int(r_st[0]["total_processed"])
    finally:
        gpu_capture.set_filter(SessionFilter.All)
        gpu_capture.set_own_ips([])
        gpu_capture.clear_all_sessions()


def test_parsed_path_matches_frame_path(gpu_capture):
    """Frames -> records, records -> parsed packets -> records again: the two GPU entry points
    agree record for record (the parsed path restates process_parsed_packet alone)."""
    from flodbadd_amd.sessions import records_to_packets
    frames, offs = synth.generate(3, 20000)
    g = gpu_capture.parse_classify(frames, offs)
    pk = records_to_packets(g.records)
    parsed = packets_to_parsed(pk)
    parsed["pkt_index"] = g.records["pkt_index"]
    gpu_capture.clear_all_sessions()
    g2 = gpu_capture.process_parsed(parsed)
    assert g2.records.tobytes() == g.records.tobytes()
    gpu_capture.clear_all_sessions()


# ---- committed golden fixtures through the GPU frame path --------------------------------------
import os  # noqa: E402

_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden(name):
    return np.load(os.path.join(_GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("tag,flt", [("all", SessionFilter.All), ("global", SessionFilter.GlobalOnly),
                                     ("local", SessionFilter.LocalOnly)])
def test_golden_edge_frames_on_gpu(gpu_capture, tag, flt):
    from flodbadd_amd.sessions import words_to_ip
    g = _golden("edge_frames.npz")
    gpu_capture.set_filter(flt)
    gpu_capture.set_lan_v6([(str(words_to_ip(r["net"], 10)), int(r["prefix"])) for r in g["lan_v6"]])
    gpu_capture.set_own_ips([str(words_to_ip(r["addr"], int(r["family"]))) for r in g["own_ips"]])
    try:
        r = gpu_capture.parse_classify(g["frames"], g["offsets"])
        assert r.records.tobytes() == g["records_" + tag].tobytes()
        assert r.dns.tobytes() == g["dns_" + tag].tobytes()
        assert np.array_equal(r.cls, g["cls_" + tag])
        st = g["stats_" + tag][0]
        for k in ("total_processed", "tcp_processed", "udp_processed", "ipv4_processed", "ipv6_processed",
                  "n_session", "n_dns", "n_drop", "n_filtered", "bad_offsets"):
            assert r.stats[k] == int(st[k]), k
    finally:
        gpu_capture.set_filter(SessionFilter.All)
        gpu_capture.set_lan_v6([])
        gpu_capture.set_own_ips([])


@pytest.mark.parametrize("cid", [2, 3])
def test_golden_samples_on_gpu(gpu_capture, cid):
    g = _golden("c%d_sample.npz" % cid)
    gpu_capture.clear_all_sessions()
    r = gpu_capture.process_frames(g["frames"], g["offsets"])
    assert r.records.tobytes() == g["records_all"].tobytes()
    assert r.dns.tobytes() == g["dns_all"].tobytes()
    assert rows_sorted(gpu_capture.export_flows()) == rows_sorted(g["flows_all"])
    assert r.stats["new_sessions"] == int(g["flow_stats_all"][0]["new_sessions"])
    gpu_capture.clear_all_sessions()
