"""Time the C5 global session table (flodbadd_amd.distributed.global_flow_table) over RCCL at world
size 1 on the device: the C4 10M-frame table (1.45M flows) exported by the library into a device
tensor grouped by owner (fb_flow_export_merge_dev), then merged by the library (fb_flow_merge_dev);
at W = 1 the two collectives are skipped.  Timed with the merged table left on the device
(as_tensor=True) and, separately, with the download to host records; --profile adds a per-kernel
torch profile of one merge."""
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

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29541"))
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
for n in (1 << 20, 10 << 20):
    frames, offs = synth.generate(4, n, first=1)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 21)
    cap.process_frames(frames, offs)
    flows = cap.flow_count()
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        merged = global_flow_table(dist, cap.ctx, device=dev, as_tensor=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        host = global_flow_table(dist, cap.ctx, device=dev)
        t2 = time.perf_counter()
        assert host.view(np.uint8).tobytes() == merged.cpu().numpy().view(np.uint8).tobytes()
        assert len(host) == flows
        print("frames %d flows %d: export + merge %.2f ms on the device, %.2f ms with the download"
              % (n, int(merged.shape[0]), (t1 - t0) * 1e3, (t2 - t1) * 1e3))
    if n == (10 << 20) and "--profile" in sys.argv:
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            global_flow_table(dist, cap.ctx, device=dev, as_tensor=True)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
    cap.close()
dist.destroy_process_group()
