"""N>1 path on the CPU (gloo, world size 2): packet-index sharding and the global per-flow
counter merge of flodbadd_amd.distributed (the C5 exchange).  The per-rank flow tables come
from the CPU oracle, standing in for each rank's GPU table (no GPU here); the code under test is
the shard arithmetic and the all-gather / dense-id / all-reduce merge, checked against the
single-process table of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from flodbadd_amd import _native as N
from flodbadd_amd.distributed import global_flow_table, shard_range, sort_keys, _key_words

TOTAL = 30000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_flows(rank, world):
    from flodbadd_amd import synth
    from oracle import coracle
    first, count = shard_range(TOTAL, rank, world)
    frames, offs = synth.generate(4, count, first=first)
    out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    fl = coracle.Flows()
    fl.update(out)
    return fl.export_sorted(), first


def _worker(rank, world, port, outdir, empty_rank=-1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        flows, first = _rank_flows(rank, world)
        if rank == empty_rank:
            flows = flows[:0]
        if rank == 1:  # the device-tensor input form (fb_flow_export_dev records), on the CPU here
            import torch
            flows = torch.from_numpy(flows.view(np.uint8).reshape(len(flows), N.FLOW_REC_DTYPE.itemsize).copy())
        merged = global_flow_table(dist, flows, shard_first=first)
        np.save(os.path.join(outdir, "r%d.npy" % rank), merged.view(np.uint8))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    for world in (1, 2, 3, 8):
        spans = [shard_range(1001, r, world) for r in range(world)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == 1001
        assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_sort_keys_is_derived_ord():
    from oracle import coracle
    flows = _rank_flows(0, 1)[0]
    rng = np.random.default_rng(1)
    shuffled = flows[rng.permutation(len(flows))]
    assert shuffled[sort_keys(_key_words(shuffled))].tobytes() == flows.tobytes()  # oracle sorts by Ord


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 3])
def test_gloo_global_flow_table(tmp_path, world):
    """world 1 (no key met twice), 2 and 3 (uneven shards, three Ord ranges): every rank ends
    with the single-process table of the whole batch, byte for byte."""
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    ref = _rank_flows(0, 1)[0]  # whole batch, one process: counters and ordered state
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        assert got.tobytes() == ref.tobytes(), r


@pytest.mark.timeout(300)
def test_gloo_merge_with_an_empty_rank(tmp_path):
    """A rank with no flows still takes part in every collective; the result is the other rank's
    table with global positions."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), 1), nprocs=world, start_method="spawn")
    only, _ = _rank_flows(0, world)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        exp = only.copy()
        exp["slot"] = 0
        assert got.tobytes() == exp.tobytes(), r
