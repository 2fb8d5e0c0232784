"""Which host calls wait for the resident queue kernel (diagnostic): with a queue live (idle_ms
5,000), time hipMalloc, a pageable H2D upload, a D2H download and hipFree of a 1-MB buffer."""
import json
import os
import sys
import time
import ctypes as C

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=0)
lib = N.gpu_lib()
pre = N.DeviceBuffer(1 << 20)
q = C.c_void_p(lib.fb_seg_queue_create(cap.ctx, 2, 5000))
assert q
out = {}
time.sleep(0.2)
a = np.ones(1 << 20, dtype=np.uint8)
t = time.perf_counter(); pre.upload(a); out["upload_ms"] = (time.perf_counter() - t) * 1e3
t = time.perf_counter(); pre.download(np.zeros(1 << 20, dtype=np.uint8)); out["download_ms"] = (time.perf_counter() - t) * 1e3
t = time.perf_counter(); b = N.DeviceBuffer(1 << 20); out["malloc_ms"] = (time.perf_counter() - t) * 1e3
t = time.perf_counter(); b.free(); out["free_ms"] = (time.perf_counter() - t) * 1e3
t = time.perf_counter(); rc = lib.fb_seg_queue_destroy(q); out["destroy_ms"] = (time.perf_counter() - t) * 1e3
out["destroy_rc"] = rc
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}))
cap.close()
