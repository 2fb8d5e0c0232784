#!/usr/bin/env python3
"""Line-traffic model of the segmented parse (k_parse_seg) on BASELINE's C2 / C3 batches.

The PMC traffic of C3 (IMIX) is ~1.18x its algorithmic bytes (profiles/pmc_traffic.json "3"), against
~1.01x for C2.  gfx950 fetches whole 128-B lines for these reads (MI355X_MICROARCH.md: FETCH_SIZE
tallies 128-B requests at 64 B), so this model counts the distinct 128-B lines each batch's reads
touch, for three load shapes:
  product   the kernel's header loads: 3 x 16 B + 4 B + 8 B from a = (o + 10) & ~3 (load_headers1,
            flodbadd_amd/csrc/fb_parse.hip), clipped to the batch
  window    only the bytes of the fixed decode window f[12..70) the rules can read (any correct
            single-round-trip load shape reads at least these)
  protocol  only the bytes each frame's decode actually reads given its EtherType / IHL / protocol
            (ethertype .. the last L4 field used) -- reachable only with dependent loads
plus the offsets array and the record / DNS writes (written whole).  Run: python3 tools/traffic_model.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from flodbadd_amd import synth  # noqa: E402
from oracle import coracle  # noqa: E402


def lines(lo, hi, limit, line):
    """Distinct `line`-byte lines touched by the byte ranges [lo, hi) (clipped to [0, limit))."""
    hi = np.minimum(hi, limit)
    ok = hi > lo
    first, last = lo[ok] // line, (hi[ok] - 1) // line
    span = last - first + 1
    idx = np.repeat(first, span) + (np.arange(span.sum()) - np.repeat(np.cumsum(span) - span, span))
    return np.unique(idx).size


def model(cid, n=1 << 20, line=128):
    fr, of = synth.generate(cid, n, first=0)
    o = of[:-1].astype(np.int64)
    cap = (of[1:] - of[:-1]).astype(np.int64)
    lim = len(fr)
    a = (o + 10) & ~3
    prod = lines(np.concatenate([a, a + 56]), np.concatenate([a + 52, a + 64]), lim, line)
    window = lines(o + 12, o + np.minimum(cap, 70), lim, line)
    b = lambda k: fr[np.minimum(o + k, lim - 1)].astype(np.int64)  # noqa: E731
    v6 = ((b(12) << 8) | b(13)) == 0x86DD
    proto = np.where(v6, b(20), b(23))
    l4 = np.where(v6, 54, 14 + (b(14) & 15) * 4)
    end = np.minimum(l4 + np.where(proto == 6, 14, 8), cap)
    proto_lines = lines(o + 12, o + end, lim, line)
    out, dns, _, _ = coracle.parse_classify(coracle.make_cfg(1), fr, of)
    rest = 56 * len(out) + 16 * len(dns) + 4 * len(of)
    alg = int(np.minimum(cap, 128).sum()) + rest
    return dict(config="C%d" % cid, frames=n, algorithmic_MB=alg / 1e6,
                **{k + "_MB": (v * line + rest) / 1e6 for k, v in (("product", prod), ("window", window),
                                                                   ("protocol", proto_lines))},
                **{k + "_x": round((v * line + rest) / alg, 3) for k, v in (("product", prod), ("window", window),
                                                                           ("protocol", proto_lines))})


if __name__ == "__main__":
    for cid in (2, 3):
        print(model(cid))
