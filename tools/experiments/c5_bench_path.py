"""Exercise bench.c5_flow_reduce's RCCL branch (device export into a torch tensor, device merge)
at world size 1 on the one-GPU box -- the branch the 8-GPU driver run takes."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from flodbadd_amd import _native as N  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
lib = N.gpu_lib()
cfg = N.FbConfig()
cfg.abi_version = N.FB_ABI_VERSION
cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 24
cfg.flow_capacity = 1 << 21
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
g = dist.new_group(backend="nccl")
r = bench.c5_flow_reduce(N, lib, ctx, 10 * (1 << 20), 0, 1, dist, g, dev)
print(json.dumps(r))
assert r["global_flows"] == r["local_flows"] > 1000000
lib.fb_destroy(ctx)
dist.destroy_process_group()
