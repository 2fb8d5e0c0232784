"""BASELINE.json configs[0] -- examples/capture_sessions.rs over loopback, 10k synthetic 64-B TCP
packets.  tests/golden/c1_loopback.npz holds 10,000 frames injected on `lo` and captured back by
examples/capture_sessions.py (tools/gen_c1_fixture.sh, CAP_NET_RAW, no GPU).  On the CPU: both
oracle restatements agree on the captured batch, every frame is a loopback session under
SessionFilter.All (100 flows, both directions of each 127.0.0.1 <-> 127.0.0.1:8080 pair folded
into one canonical key), and under the reference's default GlobalOnly every one of them is
filtered -- the reason the reference example prints 0 sessions for loopback (src/capture.rs:108,
src/packets.rs:323-324).  On the GPU: the same batch through FlodbaddGpuCapture, bit-exact."""
import os
import sys

import numpy as np
import pytest

from oracle import coracle, pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _fixture():
    g = np.load(os.path.join(HERE, "golden", "c1_loopback.npz"), allow_pickle=False)
    return g["frames"], g["offsets"]


def test_c1_fixture_oracles():
    frames, offs = _fixture()
    n = len(offs) - 1
    assert n == 10000 and frames.nbytes == 64 * n
    out, dns, cls, st = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    assert len(out) == n and len(dns) == 0 and (cls == 0).all()
    assert int(st[0]["tcp_processed"]) == n and int(st[0]["ipv4_processed"]) == n
    assert (out["packet_length"] == 10).all() and (out["ip_packet_length"] == 50).all()
    flows = coracle.Flows()
    s = np.zeros(1, dtype=st.dtype)
    flows.update(out, s)
    assert flows.count() == 100 and int(s[0]["new_sessions"]) == 100
    assert int(s[0]["updated_sessions"]) == n - 100
    # the independent restatement agrees on every class and record order
    pcfg = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=2)
    classes, records, _, _ = pyoracle.run_batch(pcfg, frames, offs)
    assert classes == cls.tolist() and [r["pkt_index"] for r in records] == out["pkt_index"].tolist()
    # GlobalOnly (FlodbaddCapture::new()'s default): loopback is local, every session filtered
    g_out, _, g_cls, g_st = coracle.parse_classify(coracle.make_cfg(1), frames, offs)
    assert len(g_out) == 0 and (g_cls == 3).all() and int(g_st[0]["n_filtered"]) == n


def test_loopback_capture_tool():
    """The capture harness itself (AF_PACKET on lo); skipped without CAP_NET_RAW."""
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import capture_sessions
    try:
        frames, offs, _ = capture_sessions.capture_loopback(300, 10, timeout=5.0)
    except (PermissionError, OSError) as e:
        pytest.skip("no raw capture on lo here: %s" % e)
    assert len(offs) - 1 == 300
    expect = b"".join(capture_sessions.frame(k, 10) for k in range(300))
    assert frames.tobytes() == expect  # each injected frame captured once, in order


@pytest.mark.gpu
def test_c1_gpu():
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    from test_gpu_parity import rows_sorted
    frames, offs = _fixture()
    r_out, _, r_cls, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    flows = coracle.Flows()
    flows.update(r_out)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16)
    try:
        g = cap.process_frames(frames, offs)
        assert g.records.tobytes() == r_out.tobytes() and np.array_equal(g.cls, r_cls)
        assert rows_sorted(cap.export_flows()) == rows_sorted(flows.export_sorted())
        assert len(cap.get_sessions()) == 100  # read before clearing (the reference's stop() clears)
        cap.clear_all_sessions()
        cap.set_filter(SessionFilter.GlobalOnly)
        g2 = cap.process_frames(frames, offs)
        assert len(g2.records) == 0 and len(cap.get_sessions()) == 0
    finally:
        cap.close()
