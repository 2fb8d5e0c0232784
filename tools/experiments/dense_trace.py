"""Timeline of one k_parse_dense launch (diagnostic; needs a -DFB_DN_TRACE build in
FLODBADD_GPU_LIB): C2, 1M frames, a few warm launches, then the last launch's per-tile and
per-block times (us from the first block's start), by round (tile t is round t // G)."""
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
cid = int(os.environ.get("CONFIG", "2"))
r = bench.run_config(N, lib, ctx, cid, 1 << 20, 20, 5, 4, 0, 1, None, mode="dense")
tr = np.zeros(4 * (8192 + 1024), dtype=np.uint64)
f = lib.fb_dense_trace_last
f.argtypes = [C.c_void_p]
assert f(tr.ctypes.data) == 0
tiles = tr[:4 * 8192].reshape(8192, 4).astype(np.float64)
blocks = tr[4 * 8192:].reshape(1024, 4).astype(np.float64)
nb = int((blocks[:, 0] > 0).sum())
nt = int((tiles[:, 1] > 0).sum())
t0 = blocks[:nb, 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
done, pub, free = us(tiles[:nt, 0]), us(tiles[:nt, 1]), us(tiles[:nt, 2])
rounds = np.arange(nt) // nb
out = dict(config=cid, mpps=round((1 << 20) * 20 / r["elapsed"] / 1e6, 1), blocks=nb, tiles=nt,
           block_start_max=round(float(us(blocks[:nb, 0]).max()), 2),
           parse_end=dict(min=round(float(us(blocks[:nb, 1]).min()), 2), med=round(float(np.median(us(blocks[:nb, 1]))), 2),
                          max=round(float(us(blocks[:nb, 1]).max()), 2)),
           block_end=dict(min=round(float(us(blocks[:nb, 2]).min()), 2), med=round(float(np.median(us(blocks[:nb, 2]))), 2),
                          max=round(float(us(blocks[:nb, 2]).max()), 2)))
print(json.dumps(out))
print("round  done(min/med/max)        offset-published(min/med/max)   offset-done lag(med/max)  freed(med/max)")
for k in range(int(rounds.max()) + 1):
    m = rounds == k
    d, p_, fr = done[m], pub[m], free[m]
    print("%5d  %6.2f %6.2f %6.2f     %6.2f %6.2f %6.2f             %6.2f %6.2f            %6.2f %6.2f" % (
        k, d.min(), np.median(d), d.max(), p_.min(), np.median(p_), p_.max(), np.median(p_ - d), (p_ - d).max(),
        np.median(fr), fr.max()))
