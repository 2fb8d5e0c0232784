"""Host-side cost of each call in bench.py's timed region (C2, one 20-batch launch): event
records, the launch call, the completion spin -- to see what the 17-20 us of host time outside
the kernel are made of."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd import synth  # noqa: E402

lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 24
cfg.flow_capacity = 1 << 21
N.check(lib.fb_set_device(0))
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
n = 1 << 20
frames, offs = synth.generate(2, n)
K = 20
bufs = []
for _ in range(K):
    bufs.append((N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
                 N.DeviceBuffer(16384 * N.SEG_BYTES), N.DeviceBuffer(16384 * 4), N.DeviceBuffer(128)))
d = np.zeros(K, dtype=N.SEG_BATCH_DTYPE)
for t, (fr, of, out, seg, st) in enumerate(bufs):
    d[t] = (fr.ptr.value, frames.nbytes, of.ptr.value, n, 0, out.ptr.value, seg.ptr.value, 0, st.ptr.value)
s = N.Stream()
ev0, ev1 = N.Event(), N.Event()
rows = []
for rep in range(12):
    s.sync()
    t0 = time.perf_counter()
    ev0.record(s)
    t1 = time.perf_counter()
    rc = lib.fb_parse_classify_seg_batches_dev(ctx, d.ctypes.data, K, s.ptr)
    t2 = time.perf_counter()
    ev1.record(s)
    t3 = time.perf_counter()
    ev1.wait_spin()
    t4 = time.perf_counter()
    assert rc == 0
    ev_ms = ev0.elapsed_ms(ev1)
    rows.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t4 - t3) * 1e6, (t4 - t0) * 1e6 - ev_ms * 1e3))
r = np.median(np.array(rows[2:]), axis=0)
print("median us: ev0.record %.1f  launch call %.1f  ev1.record %.1f  spin %.1f  | wall - event time %.1f" % tuple(r))
