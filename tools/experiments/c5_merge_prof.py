"""cProfile of one C5 merge (global_flow_table, RCCL world size 1) of the C4 table: where the
host time goes."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from flodbadd_amd import synth  # noqa: E402
from flodbadd_amd.capture import FlodbaddGpuCapture  # noqa: E402
from flodbadd_amd.distributed import global_flow_table  # noqa: E402
from flodbadd_amd.sessions import SessionFilter  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29542")
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
frames, offs = synth.generate(4, 10 << 20, first=1)
cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 21)
cap.process_frames(frames, offs)
flows = cap.export_flows()
global_flow_table(dist, flows, device=dev)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
global_flow_table(dist, flows, device=dev)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
cap.close()
dist.destroy_process_group()
