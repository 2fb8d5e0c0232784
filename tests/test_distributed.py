"""N>1 path on the CPU (gloo, world sizes 1-3): packet-index sharding and the global session table
of flodbadd_amd.distributed (BASELINE configs[4]): owner-grouped export, all_to_all, owner merge,
all_gather.  The per-rank tables come from the CPU oracle (standing in for each rank's GPU table:
no GPU here), and so does the per-owner merge (orc_flows_export_merge / orc_flow_merge restate
fb_flow_export_merge_dev / fb_flow_merge_dev; tests/test_gpu_c5.py checks the device kernels
against them).  The code under test is the exchange plumbing and the merge rules, checked against
ONE table fed the same packets in global order -- over several update calls per rank, so flows
start, carry history and end in different calls and on different ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flodbadd_amd import _native as N
from flodbadd_amd.distributed import MREC_WORDS, REC_WORDS, _key_words, exchange_merge, shard_range, sort_by_ord, sort_keys

TOTAL = 9000   # frames per global batch
CALLS = 3      # update calls (global batches) per rank
POOL = 400     # flows: each is seen in every call, on every rank, with SYN / FIN / RST here and there


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(k, first, count):
    from flodbadd_amd import synth
    return synth.generate(4, count, first=k * TOTAL + first, n_flows=POOL)


def _rank_table(rank, world):
    """Rank `rank`'s table after CALLS update calls on its shard of each global batch."""
    from oracle import coracle
    first, count = shard_range(TOTAL, rank, world)
    fl = coracle.Flows()
    for k in range(CALLS):
        frames, offs = _batch(k, first, count)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
        fl.update(out)
    return fl, first


def single_table():
    """ONE table fed the global batches in order (pkt_index = the packet's index in its batch)."""
    from oracle import coracle
    fl = coracle.Flows()
    for k in range(CALLS):
        frames, offs = _batch(k, 0, TOTAL)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
        fl.update(out)
    return fl.export_sorted()


def _oracle_merge(rows):
    from oracle import coracle
    m = np.ascontiguousarray(rows.numpy()).view(N.FLOW_MREC_DTYPE).reshape(-1)
    merged = coracle.flow_merge(m)
    return torch.from_numpy(np.ascontiguousarray(merged).view(np.int64).reshape(len(merged), REC_WORDS).copy())


# Unequal global batches (a capture loop flushing every MAX_BATCH frames or every 1 ms): the last one
# a short tail whose shard is empty on the lower ranks of a 3-rank world.
SIZES = (9000, 4097, 6001, 2)
BASE = 100000  # global batch k's frames are synth frames [k * BASE, k * BASE + size)


def _sched_batch(k, first, count):
    from flodbadd_amd import synth
    return synth.generate(4, count, first=k * BASE + first, n_flows=POOL)


def _rank_table_sched(rank, world, skip_empty):
    """Rank `rank`'s table over SIZES, one update call per global batch (none for an empty shard
    when skip_empty), and its call map (global batch << 32 | shard start per call)."""
    from oracle import coracle
    fl = coracle.Flows()
    cmap = []
    for k, size in enumerate(SIZES):
        first, count = shard_range(size, rank, world)
        if count == 0 and skip_empty:
            continue
        frames, offs = _sched_batch(k, first, count)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
        fl.update(out)
        cmap.append((k << 32) | first)
    return fl, cmap


def single_table_sched():
    from oracle import coracle
    fl = coracle.Flows()
    for k, size in enumerate(SIZES):
        frames, offs = _sched_batch(k, 0, size)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
        fl.update(out)
    return fl.export_sorted()


def _worker(rank, world, port, outdir, empty_rank=-1, sched=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if sched is None:
            fl, first = _rank_table(rank, world)
            if rank == empty_rank:
                fl.clear()
            mrecs, counts = fl.export_merge(world, rank, first)
        else:
            fl, cmap = _rank_table_sched(rank, world, skip_empty=sched == "skip")
            mrecs, counts = fl.export_merge(world, rank, call_map=cmap)
        rows = torch.from_numpy(np.ascontiguousarray(mrecs).view(np.int64).reshape(len(mrecs), MREC_WORDS).copy())
        table = exchange_merge(dist, rows, counts.tolist(), _oracle_merge)
        np.save(os.path.join(outdir, "r%d.npy" % rank), table.numpy().view(np.uint8))
    finally:
        dist.destroy_process_group()


def _rows(a):
    a = sort_by_ord(a.copy())
    a["slot"] = 0
    return a


def test_shard_range_covers_batch():
    for world in (1, 2, 3, 8):
        spans = [shard_range(1001, r, world) for r in range(world)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == 1001
        assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_sort_keys_is_derived_ord():
    flows = single_table()
    rng = np.random.default_rng(1)
    shuffled = flows[rng.permutation(len(flows))]
    assert shuffled[sort_keys(_key_words(shuffled))].tobytes() == flows.tobytes()  # oracle sorts by Ord


def test_fixture_exercises_the_ordered_merge():
    """The stream must make the merge's hard cases happen: flows ended in a later call than their
    first packet, and on a rank other than their first."""
    ref = single_table()
    ended = ref[ref["end_seen"] != N.FB_SEEN_NONE]
    assert len(ended) > POOL // 2
    assert ((ended["end_seen"] >> 32) > (ended["first_seen"] >> 32)).any()
    assert len(np.unique(ended["conn_state"])) >= 3


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 3])
def test_gloo_global_flow_table(tmp_path, world):
    """Every rank ends with the single table of the whole stream (3 update calls), byte for byte:
    counters, positions, history length / set, and end_seen / end_mask / conn_state re-decided at
    the globally first FIN/RST."""
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    ref = single_table()
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        assert len(got) == len(ref), (len(got), len(ref))
        g, e = _rows(got), _rows(ref)
        bad = np.flatnonzero(g.view(np.uint8).reshape(len(g), N.FLOW_REC_DTYPE.itemsize).any(axis=1) &
                             (g.view(np.uint8).reshape(len(g), N.FLOW_REC_DTYPE.itemsize) != e.view(np.uint8).reshape(len(e), N.FLOW_REC_DTYPE.itemsize)).any(axis=1))
        assert g.tobytes() == e.tobytes(), (r, bad[:5], g[bad[:2]], e[bad[:2]])


@pytest.mark.timeout(300)
def test_gloo_merge_with_an_empty_rank(tmp_path):
    """A rank with no flows still takes part in every collective; the result is the other rank's
    table with global positions."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), 1), nprocs=world, start_method="spawn")
    from oracle import coracle
    only, first = _rank_table(0, world)
    m, _ = only.export_merge(1, 0, first)
    exp = coracle.flow_merge(m)  # world 1: every key once
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        assert _rows(got).tobytes() == _rows(exp).tobytes(), r


def test_oracle_merge_of_one_rank_is_its_table():
    """World 1: the merge returns every flow once, unchanged (positions +0, conn_state as decided)."""
    from oracle import coracle
    fl, _ = _rank_table(0, 1)
    m, counts = fl.export_merge(1, 0, 0)
    assert int(counts[0]) == len(m) == fl.count()
    merged = coracle.flow_merge(m)
    assert _rows(merged).tobytes() == _rows(fl.export_sorted()).tobytes()


def test_unequal_batches_fixture_has_an_empty_shard():
    assert shard_range(SIZES[-1], 0, 3)[1] == 0 and shard_range(SIZES[-1], 2, 3)[1] == 2
    assert len(set(SIZES)) == len(SIZES)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,sched", [(2, "skip"), (3, "skip"), (3, "call")])
def test_gloo_global_flow_table_unequal_batches(tmp_path, world, sched):
    """Global batches of different sizes and a 2-frame tail: each rank's export takes a call map
    (global batch << 32 | its shard's start, per update call; "skip": no call for an empty shard,
    "call": an empty call) and the merged table equals ONE table of the global stream, byte for
    byte (include/flodbadd_gpu.h fb_flow_export_merge_map_dev)."""
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), -1, sched), nprocs=world,
                       start_method="spawn")
    ref = single_table_sched()
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        assert len(got) == len(ref), (len(got), len(ref))
        assert _rows(got).tobytes() == _rows(ref).tobytes(), r


def test_shard_first_layout_breaks_on_unequal_batches():
    """Why the call map exists: the single shard_first layout assumes every global batch has the
    rank's shard at the same index; with unequal batches its positions (and so last_seen / end_seen)
    are wrong for rank 1."""
    from oracle import coracle
    world = 2
    recs = []
    for r in range(world):
        fl, cmap = _rank_table_sched(r, world, skip_empty=False)
        m_map, _ = fl.export_merge(1, r, call_map=cmap)
        m_old, _ = fl.export_merge(1, r, shard_range(SIZES[0], r, world)[0])
        recs.append((m_map, m_old))
    assert recs[0][0].tobytes() == recs[0][1].tobytes()  # rank 0: shard start 0 in every batch
    assert recs[1][0].tobytes() != recs[1][1].tobytes()
