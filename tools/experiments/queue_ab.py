"""Round 5 A/B of the resident queue-fed parse: the bench's queue line (C2, 1M frames per batch, 32
rotating device batches) for the library in FLODBADD_GPU_LIB, at several ring depths; plus the
same workload as one launch per batch.  Prints one JSON line."""
import ctypes as C
import json
import os
import sys

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
out = {"lib": os.path.basename(os.environ.get("FLODBADD_GPU_LIB", "product"))}
for depth, steps in ((8, 128), (32, 128), (8, 512)):
    r = bench.queue_line(N, lib, ctx, 2, 1 << 20, steps, 16, 32, depth=depth)
    out["queue_d%d_s%d" % (depth, steps)] = r["value"]
r1 = bench.run_config(N, lib, ctx, 2, 1 << 20, 64, 8, 32, 0, 1, None, mode="seg", bpl=1)
out["launch_per_batch"] = round((1 << 20) * 64 / r1["elapsed"] / 1e6, 2)
r2 = bench.run_config(N, lib, ctx, 2, 1 << 20, 160, 20, 32, 0, 1, None, mode="seg", bpl=20)
out["launch_bpl20"] = round((1 << 20) * 160 / r2["elapsed"] / 1e6, 2)
print(json.dumps(out), flush=True)
