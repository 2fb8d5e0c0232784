#!/usr/bin/env python3
"""Experiment (not product): how much of the C4 table update is the random record gather?
Runs bench.py's C4 one-stream line on the SAME frames reordered so that every table partition's
records are contiguous (a valid capture, just in partition order): K2's gathers then stream.
Usage: python3 tools/experiments/k2_local.py [--order partition|original] -- <bench args>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from flodbadd_amd import synth  # noqa: E402

M1, M2, M3 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0xFF51AFD7ED558CCD), np.uint64(0x9E3779B97F4A7C15)


def flow_hash(words):
    """fb_flow_hash (fb_internal.h flow_hash_words) over [n,10] uint32 key words, vectorised."""
    w = words.astype(np.uint64)
    h = np.full(len(w), M3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(0, 10, 2):
            h ^= w[:, j] | (w[:, j + 1] << np.uint64(32))
            h *= M1
            h ^= h >> np.uint64(31)
        h ^= h >> np.uint64(33)
        h *= M2
        h ^= h >> np.uint64(33)
    return h


orig_generate = synth.generate


def sorted_generate(config_id, n, first=0, **kw):
    frames, offs = orig_generate(config_id, n, first=first, **kw)
    if config_id != 4:
        return frames, offs
    from oracle import coracle
    out, _, _, _ = coracle.parse_classify(coracle.make_cfg(1), frames, offs)
    words = out.view(np.uint8).reshape(len(out), 56)[:, :40].copy().view(np.uint32).reshape(len(out), 10)
    words[:, 9] &= 0xFFFF
    part = np.zeros(n, dtype=np.uint64)
    part[out["pkt_index"]] = flow_hash(words) >> np.uint64(52)  # 4096 partitions (2^21 slots)
    order = np.argsort(part, kind="stable")
    lens = np.diff(offs.astype(np.int64))
    starts = offs[:-1].astype(np.int64)
    new_lens = lens[order]
    new_offs = np.zeros(n + 1, dtype=np.uint32)
    new_offs[1:] = np.cumsum(new_lens)
    idx = np.repeat(starts[order] - new_offs[:-1].astype(np.int64), new_lens) + np.arange(int(new_offs[-1]))
    print("k2_local: reordered %d frames by partition" % n, file=sys.stderr)
    return frames[idx], new_offs


if __name__ == "__main__":
    argv = sys.argv[1:]
    order = "partition"
    if argv[:1] == ["--order"]:
        order, argv = argv[1], argv[2:]
    if argv[:1] == ["--"]:
        argv = argv[1:]
    if order == "partition":
        synth.generate = sorted_generate
    sys.argv = ["bench.py"] + argv
    import bench
    bench.main()
