"""The global session table on the GPU (BASELINE configs[4]).

* The library's export and merge kernels (fb_flow_export_merge_dev, fb_flow_merge_dev,
  flodbadd_amd/csrc/fb_merge.hip) with W "ranks" as W contexts in one process: each context runs
  its packet-index shards of several global batches (one update call per batch), exports its table
  grouped by owner, each owner's groups are concatenated in rank order and merged on the device.
  The union equals ONE table fed the same packets in global order (the oracle's), byte for byte --
  including end_seen / end_mask / conn_state decided at the globally first FIN/RST -- and every
  exported group equals the oracle's restatement (orc_flows_export_merge).
* global_flow_table over RCCL (the "nccl" backend) at world size 1 on the one-GPU box: the export
  lands in a device tensor, the merge runs on it, nothing goes through the host.  World sizes 2-3
  of the exchange itself run in tests/test_distributed.py (gloo, CPU)."""
import os
import socket

import numpy as np
import pytest

from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.distributed import shard_range, sort_by_ord
from oracle import coracle

pytestmark = pytest.mark.gpu

TOTAL, CALLS, POOL = 60000, 3, 3000


def _batch(k, first, count, pool=POOL):
    return synth.generate(4, count, first=k * TOTAL + first, n_flows=pool)


def _rows(a):
    a = sort_by_ord(np.ascontiguousarray(a).copy())
    a["slot"] = 0
    return a


def _single(pool=POOL):
    fl = coracle.Flows()
    for k in range(CALLS):
        fr, of = _batch(k, 0, TOTAL, pool)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
        fl.update(out)
    return fl.export_sorted()


def _export(cap, world, rank, first):
    import ctypes as C
    lib = N.gpu_lib()
    n = cap.flow_count()
    d_out, d_cnt = N.DeviceBuffer(max(n, 1) * N.FLOW_MREC_DTYPE.itemsize), N.DeviceBuffer(8 * world)
    N.check(lib.fb_flow_export_merge_dev(cap.ctx, world, rank, first, d_out.ptr, n, d_cnt.ptr, None))
    counts = d_cnt.download(np.zeros(world, dtype=np.uint64))
    m = d_out.download(np.zeros(max(n, 1), dtype=N.FLOW_MREC_DTYPE))[: int(counts.sum())]
    d_out.free()
    d_cnt.free()
    assert int(counts.sum()) == n
    return m, counts


def _merge_dev(cap, mrecs):
    lib = N.gpu_lib()
    m = len(mrecs)
    d_in = N.DeviceBuffer(max(m, 1) * N.FLOW_MREC_DTYPE.itemsize)
    if m:
        d_in.upload(np.ascontiguousarray(mrecs))
    d_out, d_n = N.DeviceBuffer(max(m, 1) * N.FLOW_REC_DTYPE.itemsize), N.DeviceBuffer(8)
    N.check(lib.fb_flow_merge_dev(cap.ctx, d_in.ptr, m, d_out.ptr, d_n.ptr, None))
    k = int(d_n.download(np.zeros(1, dtype=np.uint64))[0])
    out = d_out.download(np.zeros(max(m, 1), dtype=N.FLOW_REC_DTYPE))[:k]
    for b in (d_in, d_out, d_n):
        b.free()
    return out


@pytest.mark.parametrize("world", [1, 2, 3])
def test_device_export_and_merge_equal_one_table(world):
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    caps = [FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16) for _ in range(world)]
    try:
        groups = []  # per rank: (mrecs, counts)
        for r, cap in enumerate(caps):
            first, count = shard_range(TOTAL, r, world)
            ref = coracle.Flows()
            for k in range(CALLS):
                fr, of = _batch(k, first, count)
                g = cap.process_frames_seg(fr, of) if k % 2 else cap.process_frames(fr, of)
                out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
                ref.update(out)
                assert g.stats["error"] == 0
            m, counts = _export(cap, world, r, first)
            em, ecounts = ref.export_merge(world, r, first)
            assert np.array_equal(counts, ecounts)
            # the same records per owner group (the library's groups are in slot order, the oracle's in Ord)
            for o in range(world):
                a = m[int(counts[:o].sum()): int(counts[: o + 1].sum())]
                b = em[int(ecounts[:o].sum()): int(ecounts[: o + 1].sum())]
                assert np.all(a["rec"]["slot"] == r)
                ka = np.ascontiguousarray(a).view(np.uint8).reshape(len(a), N.FLOW_MREC_DTYPE.itemsize)
                kb = np.ascontiguousarray(b).view(np.uint8).reshape(len(b), N.FLOW_MREC_DTYPE.itemsize)
                ka, kb = ka[np.lexsort(ka[:, :40].T[::-1])], kb[np.lexsort(kb[:, :40].T[::-1])]
                assert ka.tobytes() == kb.tobytes(), (r, o)
            groups.append((m, counts))
        merged = []
        for o in range(world):  # owner o receives every rank's group o, in rank order
            recv = np.concatenate([m[int(c[:o].sum()): int(c[: o + 1].sum())] for m, c in groups])
            got = _merge_dev(caps[o], recv)
            assert _rows(got).tobytes() == _rows(coracle.flow_merge(recv)).tobytes(), o
            # order: each key where its first received record is
            firsts = {}
            for i, x in enumerate(recv):
                firsts.setdefault(bytes(x["rec"].tobytes()[:40]), i)
            assert [firsts[bytes(x.tobytes()[:40])] for x in got] == sorted(firsts.values())
            merged.append(got)
        table = np.concatenate(merged)
        ref = _single()
        assert len(table) == len(ref)
        assert _rows(table).tobytes() == _rows(ref).tobytes()
        ended = ref[ref["end_seen"] != N.FB_SEEN_NONE]
        assert ((ended["end_seen"] >> 32) > (ended["first_seen"] >> 32)).any()  # ends in later calls
    finally:
        for c in caps:
            c.close()


def test_merge_of_many_copies_per_key():
    """Sixteen ranks' records of the same few keys (every key on every rank): sums, min / max and
    the ending rank over 16 copies, against the oracle's merge."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    world, pool = 16, 64
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 12)
    try:
        recv = []
        for r in range(world):
            first, count = shard_range(TOTAL, r, world)
            ref = coracle.Flows()
            for k in range(2):
                fr, of = synth.generate(4, count, first=k * TOTAL + first, n_flows=pool)
                out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
                ref.update(out)
            m, _ = ref.export_merge(1, r, first)
            recv.append(m)
        recv = np.concatenate(recv)
        got = _merge_dev(cap, recv)
        exp = coracle.flow_merge(recv)
        assert len(got) == len(exp) and got.tobytes() == exp.tobytes()  # same order too
    finally:
        cap.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(rank, port, out):
    """The RCCL exchange in a fresh process: its own HIP runtime state and communicator, whatever
    the test process did on the device before."""
    import torch
    import torch.distributed as dist
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import global_flow_table
    from flodbadd_amd.sessions import SessionFilter
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 18)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        for k in range(CALLS):
            fr, of = _batch(k, 0, TOTAL, pool=1 << 20)
            cap.process_frames(fr, of)
        merged = global_flow_table(dist, cap.ctx, device=torch.device("cuda", 0))
        np.save(out, merged.view(np.uint8))
    finally:
        dist.destroy_process_group()
        cap.close()


def test_rccl_world1_global_flow_table(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "merged.npy")
    mp.start_processes(_child, args=(_free_port(), out), nprocs=1, start_method="spawn")
    merged = np.load(out).view(N.FLOW_REC_DTYPE)
    ref = _single(pool=1 << 20)
    assert len(merged) == len(ref) and _rows(merged).tobytes() == _rows(ref).tobytes()


# Unequal global batches and a 1-frame tail (rank 0's shard of it is empty: it makes no call for it).
SIZES = (60000, 20001, 35555, 1)
BASE = 1 << 20


def _sched_batch(k, first, count):
    return synth.generate(4, count, first=k * BASE + first, n_flows=POOL)


def _gloo_child(rank, world, port, outdir, layout):
    """Rank `rank` of a gloo group on GPU 0: its own context parses + upserts its shards on the
    device, then global_flow_table runs the library's export / merge kernels (the collectives move
    the records through host memory)."""
    import torch
    import torch.distributed as dist
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import call_map_entry, global_flow_table
    from flodbadd_amd.sessions import SessionFilter
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16)
    try:
        if layout == "equal":
            first, count = shard_range(TOTAL, rank, world)
            for k in range(CALLS):
                fr, of = _batch(k, first, count)
                g = cap.process_frames_seg(fr, of) if k % 2 else cap.process_frames(fr, of)
                assert g.stats["error"] == 0
            merged = global_flow_table(dist, cap.ctx, shard_first=first)
        else:
            cmap = []
            for k, size in enumerate(SIZES):
                first, count = shard_range(size, rank, world)
                if count == 0:
                    continue  # no call for an empty shard: the call map skips the batch
                fr, of = _sched_batch(k, first, count)
                g = cap.process_frames(fr, of) if k % 2 else cap.process_frames_seg(fr, of)
                assert g.stats["error"] == 0
                cmap.append(call_map_entry(k, first))
            merged = global_flow_table(dist, cap.ctx, call_map=cmap)
        np.save(os.path.join(outdir, "r%d.npy" % rank), merged.view(np.uint8))
    finally:
        cap.close()
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("layout", ["equal", "unequal"])
def test_two_process_gloo_device_merge(tmp_path, layout):
    """Two processes (ranks of a gloo group, both on GPU 0): the device export (fb_flow_export_merge_dev,
    or fb_flow_export_merge_map_dev for unequal batches and a short tail batch) and the device merge
    (fb_flow_merge_dev) through flodbadd_amd.distributed.global_flow_table.  Both ranks' tables equal
    ONE oracle table fed the same packets in global order, byte for byte."""
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_gloo_child, args=(world, _free_port(), str(tmp_path), layout), nprocs=world,
                       start_method="spawn")
    if layout == "equal":
        ref = _single()
    else:
        fl = coracle.Flows()
        for k, size in enumerate(SIZES):
            fr, of = _sched_batch(k, 0, size)
            out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
            fl.update(out)
        ref = fl.export_sorted()
    assert shard_range(SIZES[-1], 0, world)[1] == 0  # (the fixture's empty shard)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        assert len(got) == len(ref), (r, len(got), len(ref))
        assert _rows(got).tobytes() == _rows(ref).tobytes(), r


def _routed_child(rank, world, port, outdir):
    """Rank `rank` of a gloo group on GPU 0 with a TIMED context: each global batch of SIZES is parsed
    shard by shard, every record routed to its key's owner (fb_route_records_dev) and applied there
    with its capture time (flodbadd_amd.distributed.RoutedSessionTable)."""
    import torch
    import torch.distributed as dist
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import RoutedSessionTable
    from flodbadd_amd.sessions import SessionFilter
    from test_gpu_timed import frame_times
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16, timed=True)
    try:
        rt = RoutedSessionTable(dist, cap)
        for k, size in enumerate(SIZES):
            first, count = shard_range(size, rank, world)
            fr, of = _sched_batch(k, first, count)
            ts = frame_times(size, seed=50 + k, call=k)[first: first + count]
            rt.process(fr, of, first, size, ts=ts)
        flows, times = rt.global_table(with_times=True)
        np.save(os.path.join(outdir, "f%d.npy" % rank), flows.view(np.uint8))
        np.save(os.path.join(outdir, "t%d.npy" % rank), times.view(np.uint8))
    finally:
        cap.close()
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_process_routed_timed_global_table(tmp_path):
    """The routed global table (records to their key's owner before the update) on timed contexts,
    two processes over gloo: with unequal batches and an empty shard, every rank's gathered table --
    counters, positions, history length / set, conn_state and every capture-time field incl. the
    5-s segment timeout -- equals ONE timed oracle table fed the global stream, byte for byte."""
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_timed import frame_times
    world = 2
    mp.start_processes(_routed_child, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    fl = coracle.Flows()
    for k, size in enumerate(SIZES):
        fr, of = _sched_batch(k, 0, size)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
        fl.update(out, ts=frame_times(size, seed=50 + k, call=k))
    er, et = fl.export_sorted(), fl.export_times()
    for r in range(world):
        got = np.load(os.path.join(tmp_path, "f%d.npy" % r)).view(N.FLOW_REC_DTYPE)
        gt = np.load(os.path.join(tmp_path, "t%d.npy" % r)).view(N.FLOW_TIME_DTYPE)
        assert len(got) == len(er) == len(gt), (r, len(got), len(er))
        order = np.lexsort(np.ascontiguousarray(got).view(np.uint8).reshape(len(got), -1)[:, :40].T[::-1])
        got, gt = got[order], gt[order]
        eo = np.lexsort(np.ascontiguousarray(er).view(np.uint8).reshape(len(er), -1)[:, :40].T[::-1])
        e_r, e_t = er[eo], et[eo]
        got = got.copy()
        got["slot"] = 0
        e_r = e_r.copy()
        e_r["slot"] = 0
        gt = gt.copy()
        gt["slot"] = 0
        assert got.tobytes() == e_r.tobytes(), r
        assert gt.tobytes() == e_t.tobytes(), r
    assert (et["segment_count"] > 0).any() and (et["end_time_ns"] != N.FB_SEEN_NONE).any()


def _rccl_routed_child(rank, port, outdir):
    """The routed table over RCCL (the "nccl" backend, device tensors) at world size 1: the record
    routing, both all_to_all_single calls with split sizes and the gathered table take the code path
    an 8-GPU run takes, in a fresh process (its own communicator)."""
    import torch
    import torch.distributed as dist
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import RoutedSessionTable
    from flodbadd_amd.sessions import SessionFilter
    from test_gpu_timed import frame_times
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16, timed=True)
    try:
        rt = RoutedSessionTable(dist, cap, device=dev)
        for k, size in enumerate(SIZES):
            fr, of = _sched_batch(k, 0, size)
            rt.process(fr, of, 0, size, ts=frame_times(size, seed=50 + k, call=k))
        flows, times = rt.global_table(with_times=True)
        np.save(os.path.join(outdir, "f.npy"), flows.view(np.uint8))
        np.save(os.path.join(outdir, "t.npy"), times.view(np.uint8))
    finally:
        cap.close()
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_world1_routed_timed_table(tmp_path):
    """RoutedSessionTable over RCCL at world size 1 (device tensors through all_to_all_single with
    split sizes): the gathered table and its capture-time records equal the timed oracle's."""
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_timed import frame_times
    mp.start_processes(_rccl_routed_child, args=(_free_port(), str(tmp_path)), nprocs=1, start_method="spawn")
    fl = coracle.Flows()
    for k, size in enumerate(SIZES):
        fr, of = _sched_batch(k, 0, size)
        out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
        fl.update(out, ts=frame_times(size, seed=50 + k, call=k))
    er, et = fl.export_sorted(), fl.export_times()
    got = np.load(os.path.join(tmp_path, "f.npy")).view(N.FLOW_REC_DTYPE)
    gt = np.load(os.path.join(tmp_path, "t.npy")).view(N.FLOW_TIME_DTYPE)
    assert len(got) == len(er) == len(gt), (len(got), len(er))
    key = lambda a: np.lexsort(np.ascontiguousarray(a).view(np.uint8).reshape(len(a), -1)[:, :40].T[::-1])
    o, eo = key(got), key(er)
    got, gt, e_r, e_t = got[o].copy(), gt[o].copy(), er[eo].copy(), et[eo]
    got["slot"] = 0
    gt["slot"] = 0
    e_r["slot"] = 0
    assert got.tobytes() == e_r.tobytes()
    assert gt.tobytes() == e_t.tobytes()
