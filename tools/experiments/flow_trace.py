"""Per-workgroup timing of the session-table update's K2 (k_flow_apply, one workgroup per partition)
and K1c (k_flow_combine) on the C4 workload (diagnostic; needs a -DFB_FLOW_TRACE build in
FLODBADD_GPU_LIB): one-stream fused calls (fb_process_seg_dev, table only), uniform and Zipf(1.1)
flow popularity; the last batch's trace.  Answers: is K2's time its slowest partitions' (and how
many entries / how hot a slot do they hold), and how evenly do K1c's workgroups finish."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402

os.environ["FB_BENCH_ABLATION"] = "1"
lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 24
cfg.flow_capacity = 1 << 21
cfg.flags = N.FB_CFG_FIXED_TABLE
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
f = lib.fb_flow_trace_last
f.argtypes = [C.c_void_p]
TR_PARTS = 8192
n = 10 * (1 << 20)


def q(x):
    return dict(min=round(float(x.min()), 1), p50=round(float(np.median(x)), 1),
                p90=round(float(np.percentile(x, 90)), 1), p99=round(float(np.percentile(x, 99)), 1),
                max=round(float(x.max()), 1))


for name, kw in (("uniform", None), ("zipf1.1", dict(zipf=1, zipf_s=1.1))):
    r = bench.run_config(N, lib, ctx, 4, n, 4, 2, 1, 0, 1, None, flow=True, mode="seg", synth_kw=kw,
                         stage_extras=False, records=False)
    tr = np.zeros(4 * TR_PARTS + 12 * 1024, dtype=np.uint64)
    assert f(tr.ctypes.data) == 0
    k2 = tr[:4 * TR_PARTS].reshape(TR_PARTS, 4)
    k2 = k2[k2[:, 0] > 0]
    t0 = float(k2[:, 0].min())
    start = (k2[:, 0] - t0) / 100.0
    loop_end = (k2[:, 1].astype(np.float64) - t0) / 100.0
    end = (k2[:, 2] - t0) / 100.0
    dur = end - start
    ent = (k2[:, 3] & 0xFFFFFFFF).astype(np.int64)
    hmax = (k2[:, 3] >> 32).astype(np.int64)
    order = np.argsort(-end)
    slow = [dict(part=int(i), start_us=round(float(start[i]), 1), dur_us=round(float(dur[i]), 1),
                 loop_us=round(float(loop_end[i] - start[i]), 1), entries=int(ent[i]), hot_slot_chars=int(hmax[i]))
            for i in order[:8]]
    # list scheduling of the measured durations over 512 workgroup slots (two per CU): in partition
    # order (the launch's; checks the model against the span) and longest first
    def makespan(durs, slots=512):
        import heapq
        h = [0.0] * slots
        for d in durs:
            t = heapq.heappop(h)
            heapq.heappush(h, t + float(d))
        return round(max(h), 1)
    sched = dict(sum_dur_us=round(float(dur.sum()), 1), work_per_slot_us=round(float(dur.sum()) / 512, 1),
                 model_partition_order_us=makespan(dur), model_longest_first_us=makespan(np.sort(dur)[::-1]))
    k1c = tr[4 * TR_PARTS:].reshape(1024, 12)
    k1c = k1c[k1c[:, 0] > 0]
    out = dict(workload=name, step_ms=round(r["elapsed"] * 1e3 / 4, 3), flow_ms=round(r["stage"]["flow_ms"], 4),
               k2=dict(parts=int(len(k2)), span_us=round(float(end.max()), 1),
                       start_spread_us=round(float(start.max()), 1), dur_us=q(dur), entries=q(ent.astype(np.float64)),
                       hot_slot_chars=q(hmax.astype(np.float64)),
                       corr_dur_entries=round(float(np.corrcoef(dur, ent)[0, 1]), 3),
                       corr_dur_hotslot=round(float(np.corrcoef(dur, hmax)[0, 1]), 3), sched=sched, last_to_end=slow))
    if len(k1c):
        c0 = float(k1c[:, 0].min())
        ce = (k1c[:, 1] - c0) / 100.0
        out["k1c"] = dict(workgroups=int(len(k1c)), span_us=round(float(ce.max()), 1), end_us=q(ce),
                          start_spread_us=round(float((k1c[:, 0].max() - c0) / 100.0), 1),
                          groups=q(k1c[:, 2].astype(np.float64)), records=q(k1c[:, 3].astype(np.float64)),
                          groups_total=int(k1c[:, 2].sum()), records_total=int(k1c[:, 3].sum()),
                          # mean us per workgroup in each phase of its groups
                          phases_us={nm: round(float(k1c[:, 4 + i].mean()) / 100.0, 1) for i, nm in enumerate(
                              ("fetch", "init", "reduce", "number", "bitmap", "pack", "combined"))})
    print(json.dumps(out), flush=True)
