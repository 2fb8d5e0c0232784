#!/usr/bin/env python3
"""Experiment (GPU box, not product): does the C4 step overlap with itself across streams?
Two contexts (two session tables) take alternate 10M-frame C4 batches on two streams; compare the
aggregate rate with one context on one stream.  If the parse (HBM-bound) of one batch overlaps the
table update (instruction-bound) of the other, the two-stream rate is higher -- the case for a
pipelined fb_process_seg_dev."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd import synth  # noqa: E402

lib = N.gpu_lib()
N.check(lib.fb_set_device(0))
n = 10 * (1 << 20)
frames, offs = synth.generate(4, n)
nseg = (n + 63) // 64


def make_ctx():
    cfg = N.FbConfig()
    cfg.abi_version = N.FB_ABI_VERSION
    cfg.filter = N.FB_FILTER_GLOBAL_ONLY
    cfg.max_batch_packets = 1 << 24
    cfg.flow_capacity = 1 << 21
    c = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
    assert c.value, lib.fb_last_error()
    return c


d_fr = N.DeviceBuffer(frames.nbytes).upload(frames)
d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
ctxs = [make_ctx(), make_ctx()]
streams = [N.Stream(), N.Stream()]
outs = [(N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize))
        for _ in range(2)]


def step(k, i):
    o, sg, st = outs[k]
    N.check(lib.fb_process_seg_dev(ctxs[k], d_fr.ptr, frames.nbytes, d_off.ptr, n, o.ptr, sg.ptr, None, st.ptr,
                                   streams[k].ptr))


def run(nctx, steps):
    for i in range(4):
        step(i % nctx, i)
    for s in streams:
        s.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i % nctx, i)
    for s in streams:
        s.sync()
    return n * steps / (time.perf_counter() - t0) / 1e6


res = {}
for rep in range(2):
    res["one_ctx_one_stream_%d" % rep] = round(run(1, 40), 1)
    res["two_ctx_two_streams_%d" % rep] = round(run(2, 40), 1)
print(json.dumps(dict(unit="Mpackets/s", **res)))
