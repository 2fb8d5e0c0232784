"""Time fb_parse_classify_dev on one 1M-frame C2 batch with the look-back fallback forced
(FB_DENSE_STEAL_POLLS=0: every late predecessor tile recomputed) against the default, to show the
forced path really runs (tests/test_gpu_dense.py checks its outputs)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd import synth  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

frames, offs = synth.generate(2, 1 << 20, first=3)
n = len(offs) - 1
lib = N.gpu_lib()
d_fr, d_of = N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs)
d_out, d_dns, d_st = N.DeviceBuffer(n * 56), N.DeviceBuffer(n * 16), N.DeviceBuffer(128)
for polls in ("4096", "0"):
    os.environ["FB_DENSE_STEAL_POLLS"] = polls
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
    s = N.Stream()
    call = lambda: N.check(lib.fb_parse_classify_dev(cap.ctx, d_fr.ptr, frames.nbytes, d_of.ptr, n, d_out.ptr, d_dns.ptr,
                                                    None, d_st.ptr, s.ptr))
    for _ in range(5):
        call()
    s.sync()
    e0, e1 = N.Event(), N.Event()
    e0.record(s)
    for _ in range(20):
        call()
    e1.record(s)
    s.sync()
    st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
    print("steal_polls=%s: %.1f us per 1M-frame batch, n_session %d, error %d" %
          (polls, e0.elapsed_ms(e1) * 1e3 / 20, int(st[0]["n_session"]), int(st[0]["error"])))
    cap.close()
