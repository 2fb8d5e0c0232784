"""Diagnostic (not product): time the synchronous host-memory path fb_parse_classify and the
device-resident dense path per call at C2 size."""
import ctypes as C
import sys
import time

import numpy as np

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flodbadd_amd import _native as N
from flodbadd_amd import synth
import bench

lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 24
cfg.flow_capacity = 1 << 21
N.check(lib.fb_set_device(0))
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
frames, offs = synth.generate(2, 1 << 20)
print(bench.host_inclusive(N, lib, ctx, frames, offs, calls=5))
n = len(offs) - 1
d_fr = N.DeviceBuffer(frames.nbytes).upload(frames)
d_of = N.DeviceBuffer(offs.nbytes).upload(offs)
d_out = N.DeviceBuffer(n * 56)
d_dns = N.DeviceBuffer(n * 16)
d_st = N.DeviceBuffer(128)
s = N.Stream()
for label, strm in (("null", None), ("stream", s.ptr)):
    for k in range(3):
        t0 = time.perf_counter()
        N.check(lib.fb_parse_classify_dev(ctx, d_fr.ptr, frames.nbytes, d_of.ptr, n, d_out.ptr, d_dns.ptr, None, d_st.ptr, strm))
        t1 = time.perf_counter()
        if strm is None:
            N.check(lib.fb_stream_sync(None))
        else:
            s.sync()
        t2 = time.perf_counter()
        print(label, "call %.1f us, call+sync %.1f us" % ((t1 - t0) * 1e6, (t2 - t0) * 1e6))
lib.fb_destroy(ctx)
