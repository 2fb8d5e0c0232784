"""Profiling helper (GPU box): bench.py's single_batch_queue_table leg alone on a C2-style context
(fixed 2^21 table), so a kernel trace shows the update kernels beside the resident parse."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from flodbadd_amd import _native as N
    lib = N.gpu_lib()
    cfg = N.FbConfig()
    cfg.abi_version = N.FB_ABI_VERSION
    cfg.filter = N.FB_FILTER_GLOBAL_ONLY
    cfg.max_batch_packets = 1 << 24
    cfg.flow_capacity = 1 << 21
    cfg.flags = N.FB_CFG_FIXED_TABLE
    ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    print(json.dumps(bench.queue_table_line(N, lib, ctx, steps=steps, warmup=4)))
    lib.fb_destroy(ctx)


if __name__ == "__main__":
    main()
