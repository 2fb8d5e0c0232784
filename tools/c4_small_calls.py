"""Profiling helper (GPU box): the C4 mix through fb_process_seg_async_dev (table-only, pipelined,
two rotating buffer sets) at a given frames-per-call, timed over `--calls` calls after a warm-up --
the shape of bench.py's extra.c4_1m, without the other legs, so a rocprofv3 kernel trace of it shows
the per-call kernels alone.  Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--zipf", type=float, default=None)
    ap.add_argument("--sync", action="store_true", help="fb_process_seg_dev (one stream) instead of the async call")
    ap.add_argument("--timed", action="store_true", help="a timed context (FB_CFG_TIMED) with per-frame capture times")
    args = ap.parse_args()
    from flodbadd_amd import _native as N
    from flodbadd_amd import synth
    lib = N.gpu_lib()
    cfg = N.FbConfig()
    cfg.abi_version = N.FB_ABI_VERSION
    cfg.filter = N.FB_FILTER_GLOBAL_ONLY
    cfg.max_batch_packets = args.frames
    cfg.flow_capacity = 1 << 21
    cfg.flags = N.FB_CFG_FIXED_TABLE | (N.FB_CFG_TIMED if args.timed else 0)
    ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
    kw = dict(zipf=1, zipf_s=args.zipf) if args.zipf else {}
    n = args.frames
    fr, of = synth.generate(4, n, **kw)
    nseg = (n + 63) // 64
    sets = [(N.DeviceBuffer(fr.nbytes).upload(fr), N.DeviceBuffer(of.nbytes).upload(of), N.DeviceBuffer(nseg * N.SEG_BYTES),
             N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize)) for _ in range(2)]
    N.check(lib.fb_set_session_records(ctx, 0))
    s = N.Stream()
    tsb = [N.DeviceBuffer(8 * n).upload((1_700_000_000 * 10 ** 9 + j * 10 ** 9 + 2000 * np.arange(n, dtype=np.uint64))
                                        .astype(np.uint64)) for j in range(2)] if args.timed else None

    def call(i):
        b = sets[i & 1]
        if tsb:
            N.check(lib.fb_set_frame_times(ctx, tsb[i & 1].ptr))
        fn = lib.fb_process_seg_dev if args.sync else lib.fb_process_seg_async_dev
        N.check(fn(ctx, b[0].ptr, fr.nbytes, b[1].ptr, n, b[2].ptr, b[3].ptr, None, b[4].ptr, s.ptr))
    for i in range(args.warmup):
        call(i)
    N.check(lib.fb_flow_join(ctx, s.ptr))
    s.sync()
    t0 = time.perf_counter()
    for i in range(args.calls):
        call(i)
    N.check(lib.fb_flow_join(ctx, s.ptr))
    s.sync()
    el = time.perf_counter() - t0
    st = sets[0][4].download(np.zeros(1, dtype=N.STATS_DTYPE))
    print(json.dumps(dict(frames_per_call=n, calls=args.calls, Mpackets_s=round(n * args.calls / el / 1e6, 1),
                          us_per_call=round(el / args.calls * 1e6, 1), error=int(st[0]["error"]),
                          n_session=int(st[0]["n_session"]))))
    lib.fb_destroy(ctx)


if __name__ == "__main__":
    main()
