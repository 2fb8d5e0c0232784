"""Round 5 diagnostic: does a submitted batch complete in the resident queue kernel, and do host copies /
memsets issued while the queue lives complete?  Prints timings (not a test)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd import synth  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

lib = N.gpu_lib()
cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
frames, offs = synth.generate(2, 4096)
n = len(offs) - 1
fr, of = N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs)
out, seg, st = N.DeviceBuffer(64 * 56 * 64), N.DeviceBuffer(64 * 4), N.DeviceBuffer(128)
d = np.zeros(1, dtype=N.SEG_BATCH_DTYPE)
d[0] = (fr.ptr.value, frames.nbytes, of.ptr.value, n, 0, out.ptr.value, seg.ptr.value, 0, st.ptr.value)
scratch = N.DeviceBuffer(1 << 20)
q = C.c_void_p(lib.fb_seg_queue_create(cap.ctx, 4, 2000))
print("created", q.value, flush=True)
t = C.c_uint64()
for k in range(3):
    t0 = time.perf_counter()
    N.check(lib.fb_seg_queue_submit(q, N.ptr(d), C.byref(t)))
    rc = 1
    while rc == 1 and time.perf_counter() - t0 < 1.0:
        rc = lib.fb_seg_queue_query(q, t.value)
    print("batch %d: rc %d after %.3f ms; %s" % (k, rc, (time.perf_counter() - t0) * 1e3,
                                                  lib.fb_last_error().decode() if rc < 0 else ""), flush=True)
    t1 = time.perf_counter()
    s = st.download(np.zeros(1, dtype=N.STATS_DTYPE))
    print("   stats n_session %d total %d (download %.3f ms)" % (int(s[0]["n_session"]), int(s[0]["total_processed"]),
                                                               (time.perf_counter() - t1) * 1e3), flush=True)
t0 = time.perf_counter()
scratch.upload(np.zeros(1 << 20, dtype=np.uint8))
print("H2D 1 MiB while the queue lives: %.3f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
t0 = time.perf_counter()
scratch.memset(0)
N.check(lib.fb_stream_sync(None))
print("memset 1 MiB while the queue lives: %.3f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
t0 = time.perf_counter()
print("destroy rc", lib.fb_seg_queue_destroy(q), "%.3f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
