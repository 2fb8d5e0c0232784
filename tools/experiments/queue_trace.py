"""Per-batch timeline of the queue-fed parse (diagnostic; needs a -DFB_QUEUE_TRACE build in
FLODBADD_GPU_LIB).  Runs bench.queue_line's workload and prints, over the timed batches, medians
(us) of: batch-to-batch completion interval, publish -> first block, first block -> first block
done, first block done -> last block done, publish(k) - done(k - depth), and per-batch counts of
waves that drained and blocked, and host polls."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

lib = N.gpu_lib()
depth = int(os.environ.get("QDEPTH", "8"))
cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.GlobalOnly, flow_capacity=0)
steps, warm = 256, 16
r = bench.queue_line(N, lib, cap.ctx, 2, 1 << 20, steps, warm, 32, depth=depth)
f = lib.fb_seg_queue_trace_last
f.argtypes = [C.c_void_p]
tr = np.zeros(6 * 1024 + 4 * 1024, dtype=np.uint64)
f(tr.ctypes.data)
blk = tr[6 * 1024:].reshape(1024, 4)
tr = tr[:6 * 1024].reshape(6, 1024).astype(np.float64)
pub, first, arr0, done, drain, polls = tr
ks = np.arange(warm + 1, warm + steps)  # batches of the timed region (ticket warm-1 ended the warmup)
us = 0.01  # 100-MHz ticks -> us


def med(x):
    return round(float(np.median(x)), 2)


out = dict(lib=os.path.basename(os.environ.get("FLODBADD_GPU_LIB", "")), depth=depth, mpps=r["value"],
           interval=med(np.diff(done[ks]) * us), pub_to_first=med((first[ks] - pub[ks]) * us),
           first_to_arr0=med((arr0[ks] - first[ks]) * us), arr0_to_done=med((done[ks] - arr0[ks]) * us),
           first_to_done=med((done[ks] - first[ks]) * us),
           pub_after_done_prev=med((pub[ks] - done[ks - depth]) * us),
           drains=med(drain[ks]), drains_mean=round(float(drain[ks].mean()), 2), polls=med(polls[ks]),
           polls_mean=round(float(polls[ks].mean()), 2),
           p90_interval=round(float(np.percentile(np.diff(done[ks]) * us, 90)), 2))
print(json.dumps(out))
for k in ks[:24]:
    print(k, "pub %.1f first %.1f arr0 %.1f done %.1f drain %d polls %d" % (
        (pub[k] - pub[ks[0]]) * us, (first[k] - pub[ks[0]]) * us, (arr0[k] - pub[ks[0]]) * us,
        (done[k] - pub[ks[0]]) * us, drain[k], polls[k]))
# per block: its rate over batches 100..164 and where it ran (HW_ID: cu bits 11:8, sh 12, se 15:13 (gfx9);
# XCC_ID low bits)
used = blk[:, 0] > 0
b = blk[used]
rate = (b[:, 1].astype(np.float64) - b[:, 0]) * us / 64.0
hw, xcc = b[:, 2].astype(np.int64), b[:, 3].astype(np.int64) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
place = xcc * 1000 + se * 100 + sh * 16 + cu
uniq, inv, cnt = np.unique(place, return_inverse=True, return_counts=True)
per_cu = cnt[inv]
print(json.dumps(dict(blocks=int(used.sum()), cus=int(len(uniq)), blocks_per_cu_hist={int(k): int((cnt == k).sum()) for k in np.unique(cnt)},
                      rate_us_per_batch=dict(min=round(float(rate.min()), 2), med=med(rate), max=round(float(rate.max()), 2)),
                      rate_by_cu_load={int(k): med(rate[per_cu == k]) for k in np.unique(per_cu)},
                      rate_by_xcc={int(x): med(rate[xcc == x]) for x in np.unique(xcc)})))
cap.close()
