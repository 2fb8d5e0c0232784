#!/usr/bin/env python3
"""GPU box: only the DNS divert parse timing of bench.py (1M synthetic port-53 payloads), for
kernel traces / PMC passes of k_dns_parse alone."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402

lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 20
cfg.flow_capacity = 1 << 16
N.check(lib.fb_set_device(0))
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
stream = N.Stream()
print(json.dumps(bench.dns_timing(N, lib, ctx, stream, reps=int(os.environ.get("REPS", "10")))))
lib.fb_destroy(ctx)
