"""GPU parse + classify on mutated frames (tests/fuzzframes.py: header bytes, truncations,
EtherTypes, IHL / lengths / next header, TCP data offset and flags, port 53, LAN addresses, pure
random bytes) against the C oracle, bit-exact under each filter with IPv6 LAN prefixes and own IPs
configured: dense records, DNS side records, classes and stats; the segmented path's records and
the session table after two batches."""
import numpy as np
import pytest

import fuzzframes
from flodbadd_amd.capture import FlodbaddGpuCapture, lan_v6_table, own_ip_table
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle
from test_gpu_parity import _assert_same, rows_sorted

pytestmark = pytest.mark.gpu

LAN = [("fd12::", 16), ("2001:db8:abcd:12::1", 64)]
OWN = ["10.0.0.1", "192.168.1.7", "fe80::1"]


@pytest.fixture(scope="module")
def fuzz_batches():
    return [fuzzframes.generate(100000, seed=101 + k) for k in range(2)]


@pytest.mark.parametrize("flt", [SessionFilter.All, SessionFilter.GlobalOnly, SessionFilter.LocalOnly])
def test_fuzz_dense_and_segmented(fuzz_batches, flt):
    cap = FlodbaddGpuCapture(0, session_filter=flt, flow_capacity=1 << 20, lan_v6=LAN, own_ips=OWN)
    cfg = coracle.make_cfg(int(flt), lan_v6=lan_v6_table(LAN), own_ips=own_ip_table(OWN))
    flows = coracle.Flows()
    try:
        for frames, offs in fuzz_batches:
            ref = coracle.parse_classify(cfg, frames, offs)
            _assert_same(cap.parse_classify(frames, offs), ref)
            g = cap.process_frames_seg(frames, offs)  # segmented path + session-table upsert
            assert g.records.tobytes() == ref[0].tobytes() and g.dns.tobytes() == ref[1].tobytes()
            assert np.array_equal(g.cls, ref[2])
            flows.update(ref[0])
        assert rows_sorted(cap.export_flows()) == rows_sorted(flows.export_sorted())
        assert len(ref[0]) > 0 and len(ref[1]) > 0  # sessions and DNS records on every filter
    finally:
        cap.close()
