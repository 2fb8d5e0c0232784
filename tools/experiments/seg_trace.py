"""Per-block balance of one k_parse_seg launch (diagnostic; needs a -DFB_SEG_TRACE build in
FLODBADD_GPU_LIB): C2 1M-frame batches, BPL batches per launch (default 20, the headline) and one;
per block the end of its segment loop and its segments, relative to the first block's start."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402

lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 20
cfg.flow_capacity = 0
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
f = lib.fb_seg_trace_last
f.argtypes = [C.c_void_p]
for bpl in (int(os.environ.get("BPL", "20")), 1):
    r = bench.run_config(N, lib, ctx, 2, 1 << 20, 2 * bpl, bpl, 32, 0, 1, None, mode="seg", bpl=bpl)
    tr = np.zeros(4 * 2048, dtype=np.uint64)
    assert f(tr.ctypes.data) == 0
    t = tr.reshape(2048, 4).astype(np.float64)
    nb = int((t[:, 0] > 0).sum())
    t = t[:nb]
    t0 = t[:, 0].min()
    loop_end = (t[:, 1] - t0) / 100.0
    end = (t[:, 3] - t0) / 100.0
    segs = t[:, 2]
    q = lambda x: dict(min=round(float(x.min()), 2), p10=round(float(np.percentile(x, 10)), 2),  # noqa: E731
                       med=round(float(np.median(x)), 2), p90=round(float(np.percentile(x, 90)), 2),
                       max=round(float(x.max()), 2))
    print(json.dumps(dict(batches_per_launch=bpl, blocks=nb, start_spread_us=round(float((t[:, 0].max() - t0) / 100.0), 2),
                          loop_end_us=q(loop_end), end_us=q(end), segments_per_block=q(segs),
                          idle_frac=round(float(1.0 - loop_end.mean() / loop_end.max()), 4))))
