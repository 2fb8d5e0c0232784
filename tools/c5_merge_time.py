"""Time the C5 merge (flodbadd_amd.distributed.global_flow_table) over RCCL at world size 1 on the
device: the C4 10M-frame table (1.45M flows) exported into a device tensor (fb_flow_export_dev),
then merged (Ord sort of the owned records, equal keys merged, records assembled on the device;
at W = 1 the owner split and the two collectives are skipped).  Timed with the merged table left
on the device (as_tensor=True) and, separately, with the download to host records."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from flodbadd_amd import synth  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.distributed import global_flow_table  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29541")
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
for n in (1 << 20, 10 << 20):
    frames, offs = synth.generate(4, n, first=1)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 21)
    cap.process_frames(frames, offs)
    import ctypes as C
    from flodbadd_amd import _native as N
    cnt = C.c_uint64()
    N.check(N.gpu_lib().fb_flow_count(cap.ctx, C.byref(cnt), None))
    flows = torch.empty((cnt.value, N.FLOW_REC_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(1, dtype=torch.int64, device=dev)
    N.check(N.gpu_lib().fb_flow_export_dev(cap.ctx, C.c_void_p(flows.data_ptr()), cnt.value,
                                           C.c_void_p(d_n.data_ptr()), None))
    torch.cuda.synchronize()
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        merged = global_flow_table(dist, flows, device=dev, as_tensor=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        host = global_flow_table(dist, flows, device=dev)
        t2 = time.perf_counter()
        assert host.view(np.uint8).tobytes() == merged.cpu().numpy().tobytes()
        print("frames %d flows %d: merge %.2f ms on the device, %.2f ms with the download"
              % (n, int(merged.shape[0]), (t1 - t0) * 1e3, (t2 - t1) * 1e3))
    if n == (10 << 20) and "--profile" in sys.argv:  # where the merge's time goes, per torch op
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            global_flow_table(dist, flows, device=dev, as_tensor=True)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
    cap.close()
dist.destroy_process_group()
