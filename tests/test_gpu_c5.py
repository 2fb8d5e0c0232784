"""C5 exchange on the GPU: global_flow_table with device tensors over RCCL (the "nccl" backend),
world size 1 on the one-GPU box -- the union, Ord sort and dense ids run as torch ops on the
device and the all-gather / all-reduce go through RCCL.  The merged table must equal the GPU
session table of the same batch sorted by Session's derived Ord (the oracle's order).  World
size 2 runs in tests/test_distributed.py (gloo, CPU)."""
import os
import socket

import numpy as np
import pytest

from flodbadd_amd import synth
from oracle import coracle

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(rank, port, out):
    """The RCCL merge in a fresh process: its own HIP runtime state and communicator, whatever the
    test process did on the device before."""
    import torch
    import torch.distributed as dist
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import global_flow_table
    from flodbadd_amd.sessions import SessionFilter
    frames, offs = synth.generate(4, 200000, first=7)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cap.process_frames(frames, offs)
        merged = global_flow_table(dist, cap.export_flows(), device=torch.device("cuda", 0))
        np.save(out, merged.view(np.uint8))
    finally:
        dist.destroy_process_group()
        cap.close()


def test_rccl_world1_global_flow_table(tmp_path):
    import torch.multiprocessing as mp
    from flodbadd_amd import _native as N
    out = str(tmp_path / "merged.npy")
    mp.start_processes(_child, args=(_free_port(), out), nprocs=1, start_method="spawn")
    merged = np.load(out).view(N.FLOW_REC_DTYPE)
    frames, offs = synth.generate(4, 200000, first=7)
    r_out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    ref = coracle.Flows()
    ref.update(r_out)
    exp = ref.export_sorted()
    a, b = merged.copy(), exp.copy()
    a["slot"] = 0
    b["slot"] = 0
    assert len(a) == len(b) and a.tobytes() == b.tobytes()
