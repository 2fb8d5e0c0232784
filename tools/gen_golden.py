#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run here, on the CPU).

Expected outputs come from the C restatement (oracle/oracle.c) and are cross-checked, before
being written, against the independent pure-Python restatement (oracle/pyoracle.py) -- the two
were written separately from the reference sources.  Byte-level decode rules
follow pnet_packet 0.35.0 semantics, which the reference does not vendor and no reference test
exercises: those expectations are "parity unpinned" (Oracle).  The classification
stage is pinned separately by tests/golden/reference_kats.json.

Fixtures (numpy .npz, loaded with allow_pickle=False):
  edge_frames.npz     hand-built edge cases (tests/framegen.edge_cases) + expected outputs for
                      filters All / GlobalOnly / LocalOnly with an IPv6 LAN prefix and own IPs
  c2_sample.npz       4096 frames of BASELINE config C2 (64-B IPv4/TCP) + expected outputs
  c3_sample.npz       4096 frames of C3 (IMIX, v4/v6, TCP/UDP) + expected outputs + flow table
Usage: python3 tools/gen_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import framegen as fg  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd import synth  # noqa: E402
from flodbadd_amd.build import build_oracle, build_synth  # noqa: E402
from flodbadd_amd.capture import lan_v6_table, own_ip_table  # noqa: E402
from oracle import coracle, pyoracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
LAN = [("2001:db8:abcd:12::1", 64)]
OWN = ["192.168.1.1", "10.0.0.5", "2001:db8::1"]


def cross_check(flt, frames, offs, res, lan=(), own=()):
    """The C oracle's outputs == the Python restatement's, field by field."""
    out, dns, cls, st = res
    pcfg = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=flt, lan_v6=lan, own_ips=own)
    classes, records, pdns, pst = pyoracle.run_batch(pcfg, frames, offs)
    assert list(cls) == classes, "class mismatch"
    assert len(out) == len(records)
    for r, c in zip(out, records):
        row = pyoracle.record_to_row(c)
        for k, v in row.items():
            got = r[k].tolist() if hasattr(r[k], "tolist") else r[k]
            assert got == v, (k, got, v)
    assert [tuple(int(x) for x in (d["pkt_index"], d["payload_offset"], d["payload_length"], d["protocol"],
                                   d["family"])) for d in dns] == [tuple(t) for t in pdns]
    for k, v in pst.items():
        assert int(st[0][k]) == v, k


def expected(flt, frames, offs, lan=(), own=()):
    cfg = coracle.make_cfg(flt, lan_v6=lan_v6_table(list(lan)), own_ips=own_ip_table(list(own)))
    res = coracle.parse_classify(cfg, frames, offs)
    cross_check(flt, frames, offs, res, lan, own)
    return res


def flows_of(records):
    fl = coracle.Flows()
    st = np.zeros(1, dtype=N.STATS_DTYPE)
    fl.update(records, st)
    return fl.export_sorted(), st


def main():
    build_synth()
    build_oracle()
    os.makedirs(OUT, exist_ok=True)
    # ---- edge cases ----------------------------------------------------------------------
    names, frames_l = zip(*fg.edge_cases())
    frames, offs = fg.pack(list(frames_l))
    d = dict(frames=frames, offsets=offs, names=np.array(names, dtype="U64"),
             lan_v6=lan_v6_table(LAN), own_ips=own_ip_table(OWN))
    for flt, tag in ((2, "all"), (1, "global"), (0, "local")):
        out, dns, cls, st = expected(flt, frames, offs, LAN, OWN)
        d["records_" + tag], d["dns_" + tag], d["cls_" + tag], d["stats_" + tag] = out, dns, cls, st
    np.savez_compressed(os.path.join(OUT, "edge_frames.npz"), **d)
    print("edge_frames.npz: %d frames" % len(names))
    # ---- synthetic samples ---------------------------------------------------------------
    for cid in (2, 3):
        frames, offs = synth.generate(cid, 4096)
        out, dns, cls, st = expected(2, frames, offs)
        flows, fst = flows_of(out)
        gout, gdns, gcls, gst = expected(1, frames, offs)
        np.savez_compressed(os.path.join(OUT, "c%d_sample.npz" % cid), frames=frames, offsets=offs,
                            records_all=out, dns_all=dns, cls_all=cls, stats_all=st, flows_all=flows,
                            flow_stats_all=fst, records_global=gout, cls_global=gcls, stats_global=gst)
        print("c%d_sample.npz: %d frames, %d records, %d dns, %d flows" % (cid, len(offs) - 1, len(out), len(dns),
                                                                          len(flows)))


if __name__ == "__main__":
    main()
