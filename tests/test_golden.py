"""Committed golden fixtures (tests/golden/*.npz, written by tools/gen_golden.py) re-derived on
the CPU: the C oracle reproduces them byte for byte, the independent Python restatement agrees on
the edge cases, and the deterministic synthetic generator reproduces the sample batches."""
import os

import numpy as np
import pytest

from flodbadd_amd import synth
from oracle import coracle, pyoracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILTERS = {"all": 2, "global": 1, "local": 0}


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("tag", sorted(FILTERS))
def test_edge_frames_c_oracle(tag):
    g = load("edge_frames.npz")
    cfg = coracle.make_cfg(FILTERS[tag], lan_v6=g["lan_v6"], own_ips=g["own_ips"])
    out, dns, cls, st = coracle.parse_classify(cfg, g["frames"], g["offsets"])
    assert out.tobytes() == g["records_" + tag].tobytes()
    assert dns.tobytes() == g["dns_" + tag].tobytes()
    assert np.array_equal(cls, g["cls_" + tag])
    assert st.tobytes() == g["stats_" + tag].tobytes()


def test_edge_frames_python_oracle():
    g = load("edge_frames.npz")
    from flodbadd_amd.sessions import words_to_ip
    lan = [(str(words_to_ip(r["net"], 10)), int(r["prefix"])) for r in g["lan_v6"]]
    own = [str(words_to_ip(r["addr"], int(r["family"]))) for r in g["own_ips"]]
    for tag, flt in FILTERS.items():
        pcfg = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=flt, lan_v6=lan, own_ips=own)
        classes, records, dns, st = pyoracle.run_batch(pcfg, g["frames"], g["offsets"])
        assert classes == g["cls_" + tag].tolist(), tag
        assert [r["pkt_index"] for r in records] == g["records_" + tag]["pkt_index"].tolist()


def test_edge_cases_cover_every_decode_rule():
    """SURVEY.md 8a decode rules each have at least one edge frame (names from framegen)."""
    names = " ".join(load("edge_frames.npz")["names"].tolist())
    for needle in ("short", "vlan", "arp", "ihl", "tot_", "doff", "v6_", "ext_hdr", "dns_tcp_1b", "udp_len",
                   "padding", "same_ip", "lan_prefix", "version_6"):
        assert needle in names.lower(), needle


@pytest.mark.parametrize("cid", [2, 3])
def test_samples_c_oracle_and_generator(cid):
    g = load("c%d_sample.npz" % cid)
    frames, offs = synth.generate(cid, 4096)
    assert np.array_equal(frames, g["frames"]) and np.array_equal(offs, g["offsets"])
    out, dns, cls, st = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    assert out.tobytes() == g["records_all"].tobytes()
    assert dns.tobytes() == g["dns_all"].tobytes()
    assert st.tobytes() == g["stats_all"].tobytes()
    fl = coracle.Flows()
    fl.update(out)
    assert fl.export_sorted().tobytes() == g["flows_all"].tobytes()
    gout, _, gcls, gst = coracle.parse_classify(coracle.make_cfg(1), frames, offs)
    assert gout.tobytes() == g["records_global"].tobytes()


@pytest.mark.parametrize("cid", [2, 3])
def test_samples_flow_table_matches_python_restatement(cid):
    """The C oracle's session table (counters, history length, conn_state, segment state) equals the
    independent Python restatement's dict table on the sample batches."""
    g = load("c%d_sample.npz" % cid)
    fl = coracle.Flows()
    fl.update(g["records_all"])
    pcfg = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=2)
    table = pyoracle.SessionTable()
    pyoracle.run_batch(pcfg, g["frames"], g["offsets"], table)
    got = pyoracle.rows_of_flow_recs(fl.export_sorted())
    assert got == pyoracle.table_rows(table)
    segs = [v[8] for v in got.values()]
    assert sum(segs) > 0 and any(not v[9] for v in got.values())  # the mix has PSH packets
