"""Multi-GPU data path: packet-index shards, and the global session table (BASELINE configs[4]).

SURVEY.md 8e.  Decode/classify has no cross-packet state, so a batch of N*W frames shards by
contiguous packet-index range: rank r owns [r*N, (r+1)*N) and runs its own context with no
data-path collective (bench.py reports "scaling": "weak").  The one real exchange is the global
session table -- the reference's single DashMap that every capture task updates
(src/capture.rs:946-1016, src/packets.rs:329-535) -- built from the ranks' tables, O(F) per rank:
  1. every rank exports its table grouped by owner rank (fb_flow_export_merge_dev: the key's hash
     picks the owner, positions made global with the shard's first packet index, plus the update
     call of each flow's first S / s / H / h);
  2. all_to_all of the groups (RCCL over xGMI with device tensors; gloo on the CPU);
  3. each owner merges what it received (fb_flow_merge_dev, flodbadd_amd/csrc/fb_merge.hip):
     integer sums (segment_count too), MIN first_seen, MAX last_seen, hist_len SUM, hist_mask OR,
     in_segment from the latest packet's record, session flags from the earliest's, and end_seen /
     end_mask / conn_state at the globally first FIN/RST -- exact for any number of update calls
     per rank (call k of every rank = its shard of global batch k, at the same offset in each);
  4. all_gather of the merged records.
BASELINE configs[4] names an all-reduce of per-flow counters; an all-reduce needs the same dense
flow index on every rank (a dictionary step: all-gather of every rank's keys and a global sort),
and its payload is the whole F-flow counter matrix on every rank.  The owner exchange moves each
flow's record once each way instead and reduces every counter exactly once (integer sums, so the
result is bit-identical to an all-reduce), with no global sort.
Bytes per rank: 152 B x its flows out (x (W-1)/W) and ~the same in, 136 B x the global flows
gathered.
"""
import ctypes as C

import numpy as np

from ._native import FLOW_MREC_DTYPE, FLOW_REC_DTYPE

MREC_WORDS = FLOW_MREC_DTYPE.itemsize // 8  # 19 u64 words per exported record
REC_WORDS = FLOW_REC_DTYPE.itemsize // 8    # 17
assert MREC_WORDS * 8 == FLOW_MREC_DTYPE.itemsize and REC_WORDS * 8 == FLOW_REC_DTYPE.itemsize


def shard_range(total, rank, world):
    """Contiguous packet-index shard of rank `rank` (first, count); the last rank takes the rest."""
    per = total // world
    first = rank * per
    return first, (total - first if rank == world - 1 else per)


def _key_words(flows):
    """[F,10] uint32 view of the 40-byte session keys."""
    return np.ascontiguousarray(flows).view(np.uint8).reshape(len(flows), FLOW_REC_DTYPE.itemsize)[:, :40] \
        .copy().view(np.uint32).reshape(len(flows), 10)


def sort_keys(words):
    """Row order of [F,10] key words by the derived Ord of Session (src/sessions.rs:23-30)."""
    src, dst = words[:, 0:4], words[:, 4:8]
    ports, pf = words[:, 8], words[:, 9]
    sport, dport = ports & 0xFFFF, ports >> 16
    proto, fam = pf & 0xFF, (pf >> 8) & 0xFF
    cols = [dport, dst[:, 3], dst[:, 2], dst[:, 1], dst[:, 0], sport, src[:, 3], src[:, 2], src[:, 1], src[:, 0],
            fam, proto]
    return np.lexsort(cols)  # last column is the primary key


def sort_by_ord(flows):
    """FLOW_REC_DTYPE records in Session's derived Ord (the reference's session order when sorted)."""
    return flows[sort_keys(_key_words(flows))] if len(flows) else flows


def _mark(timing, dev, key, t0):
    """timing[key] += milliseconds since t0 (the device drained first for a cuda `dev`); returns now."""
    import time
    if timing is None:
        return t0
    if dev.type == "cuda":
        import torch
        torch.cuda.synchronize(dev)
    now = time.perf_counter()
    timing[key] = timing.get(key, 0.0) + (now - t0) * 1e3
    return now


def exchange_merge(dist, mrecs, counts, merge, device=None, group=None, timing=None):
    """Steps 2-4 of the global session table.  `mrecs`: this rank's exported records grouped by
    owner ([n, MREC_WORDS] int64 tensor on `device`, FLOW_MREC_DTYPE rows), `counts`: the group sizes
    (sequence of W ints); `merge(rows)` maps the [m, MREC_WORDS] int64 rows this rank received (each
    rank's group, rank order) to the merged [k, REC_WORDS] int64 FLOW_REC_DTYPE rows.  Returns the
    [G, REC_WORDS] int64 global table, owners in rank order, identical on every rank.  `timing` (a dict,
    optional): milliseconds and bytes of the collectives (a2a_ms / a2a_bytes: this rank's records sent
    to other ranks; gather_ms / gather_bytes: merged records received from other ranks) apart from the
    merge (merge_ms), each stage drained before the next is timed."""
    import time
    import torch
    dev = torch.device("cpu") if device is None else torch.device(device)
    world = dist.get_world_size(group)
    counts = [int(c) for c in counts]
    if len(counts) != world or sum(counts) != int(mrecs.shape[0]):
        raise ValueError("group sizes %s do not cover the %d exported records of %d ranks"
                         % (counts, int(mrecs.shape[0]), world))
    t0 = time.perf_counter()
    if world > 1:
        send_n = torch.tensor(counts, dtype=torch.int64, device=dev)
        recv_n = torch.empty_like(send_n)
        dist.all_to_all_single(recv_n, send_n, group=group)
        rn = recv_n.tolist()
        recv = torch.empty((sum(rn), MREC_WORDS), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv, mrecs.contiguous(), output_split_sizes=rn, input_split_sizes=counts,
                               group=group)
        if timing is not None:
            rank = dist.get_rank(group)
            timing["a2a_bytes"] = timing.get("a2a_bytes", 0) + 8 * MREC_WORDS * (sum(counts) - counts[rank])
    else:
        recv = mrecs
    t0 = _mark(timing, dev, "a2a_ms", t0)
    merged = merge(recv)
    t0 = _mark(timing, dev, "merge_ms", t0)
    if world == 1:
        return merged
    n = torch.tensor([int(merged.shape[0])], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    pad = torch.zeros((max(sizes + [1]), REC_WORDS), dtype=torch.int64, device=dev)
    pad[: merged.shape[0]] = merged
    got = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(got, pad, group=group)
    out = torch.cat([g[:sz] for g, sz in zip(got, sizes)])
    _mark(timing, dev, "gather_ms", t0)
    if timing is not None:
        timing["gather_bytes"] = timing.get("gather_bytes", 0) + 8 * REC_WORDS * (sum(sizes) - int(merged.shape[0]))
    return out


def call_map_entry(global_batch, shard_first):
    """One entry of an export call map: this rank's update call was its shard of `global_batch`,
    starting at global packet index `shard_first` of that batch."""
    return (int(global_batch) << 32) | int(shard_first)


def global_flow_table(dist, ctx, shard_first=0, device=None, group=None, as_tensor=False, stream=None, timing=None,
                      call_map=None):
    """The global session table of every rank's context `ctx` (an fb_ctx handle) on the GPU: the
    library exports the owner groups into a device tensor, RCCL moves them (`device` a cuda device
    and `group` an nccl group; gloo with CPU tensors works too, the records then go through host
    memory), the library merges each owner's records.  `shard_first`: the global index of this
    rank's first packet (shard_range) when call k of every rank was its shard of equal-size global
    batch k; `call_map` (a sequence of call_map_entry per update call of this rank) for any other
    layout -- unequal per-call batches, a short tail batch, no call for an empty shard
    (fb_flow_export_merge_map_dev).  Returns FLOW_REC_DTYPE records in owner order, or with
    as_tensor=True the [G, REC_WORDS] int64 tensor on `device` (no download).

    The library's kernels run on `stream` (None: the null stream); torch's copies and reads run on
    torch's current stream of the context's device, so each hand-over between the two synchronises
    the producing side first: the export's stream before its counts / records are read, torch's
    stream before the merge reads the received rows, the merge's stream before its count is read.
    `timing`: as exchange_merge, plus export_ms (the library's owner-grouped export and its copy to
    `device`)."""
    import time
    import torch
    from . import _native as N
    lib = N.gpu_lib()
    dev = torch.device("cpu") if device is None else torch.device(device)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    cdev = C.c_int(-1)
    N.check(lib.fb_ctx_device(ctx, C.byref(cdev)))
    gpu = torch.device("cuda", cdev.value)  # buffers on the context's device
    if dev.type == "cuda" and dev.index is not None and dev.index != gpu.index:
        raise ValueError("device %s is not the context's device %s" % (dev, gpu))

    def stream_sync():
        N.check(lib.fb_stream_sync(stream))

    t0 = time.perf_counter()
    cnt = C.c_uint64()
    N.check(lib.fb_flow_count(ctx, C.byref(cnt), stream))
    mrecs = torch.empty((max(cnt.value, 1), MREC_WORDS), dtype=torch.int64, device=gpu)
    counts = torch.zeros(world, dtype=torch.int64, device=gpu)
    torch.cuda.current_stream(gpu).synchronize()  # the buffers' allocation / zeroing before the export
    if call_map is None:
        N.check(lib.fb_flow_export_merge_dev(ctx, world, rank, int(shard_first), C.c_void_p(mrecs.data_ptr()),
                                             cnt.value, C.c_void_p(counts.data_ptr()), stream))
    else:
        cm = np.ascontiguousarray(np.asarray(list(call_map), dtype=np.uint64).reshape(-1))
        N.check(lib.fb_flow_export_merge_map_dev(ctx, world, rank, N.ptr(cm) if cm.size else None, int(cm.size),
                                                 C.c_void_p(mrecs.data_ptr()), cnt.value,
                                                 C.c_void_p(counts.data_ptr()), stream))
    stream_sync()  # the group sizes and records are complete before torch reads them
    counts = counts.tolist()  # (host ints: the collective's split sizes)
    mrecs = mrecs[: sum(counts)].to(dev)
    _mark(timing, gpu, "export_ms", t0)

    def merge(rows):
        m = int(rows.shape[0])
        src = rows.to(gpu).contiguous()
        out = torch.empty((max(m, 1), REC_WORDS), dtype=torch.int64, device=gpu)
        d_n = torch.zeros(1, dtype=torch.int64, device=gpu)
        torch.cuda.current_stream(gpu).synchronize()  # the received rows' copy lands before the merge reads it
        N.check(lib.fb_flow_merge_dev(ctx, C.c_void_p(src.data_ptr()), m, C.c_void_p(out.data_ptr()),
                                      C.c_void_p(d_n.data_ptr()), stream))
        stream_sync()  # the merged records and their count are complete
        return out[: int(d_n.item())].to(dev)

    table = exchange_merge(dist, mrecs, counts, merge, device=dev, group=group, timing=timing)
    if as_tensor:
        return table
    return np.ascontiguousarray(table.cpu().numpy()).view(FLOW_REC_DTYPE).reshape(-1)


class RoutedSessionTable:
    """The global session table with EVERY kind of session state exact -- the ordered history and
    conn_state, and on a timed context the 5-s segment timeout and capture times, whose decisions
    depend on each flow's previous packet wherever it was captured: records are routed to their key's
    owner rank BEFORE the update (fb_route_records_dev), and each owner runs one update call per global
    batch over every rank's records in rank (= global packet) order.  Owner o's table is then exactly
    the single-table state of the flows o owns; `global_table` gathers them.

    Per global batch: parse the rank's shard (fb_parse_classify_dev, dense records, no update), route
    (owner groups, pkt_index made global, capture times beside them), all_to_all of the groups (RCCL
    with device tensors, or gloo through host memory), the owner's update on what it received (frame
    times scattered into a global-batch array by pkt_index).  Bytes per rank and batch: 56 B (+8 B of
    time) per SESSION record out x (W-1)/W and about as much in -- a per-batch exchange of records,
    where the merge of global_flow_table moves each flow once at the end; the price of exact ordered
    state across ranks."""

    def __init__(self, dist, capture, group=None, device=None):
        import torch
        self.dist, self.cap, self.group = dist, capture, group
        self.dev = torch.device("cpu") if device is None else torch.device(device)
        cdev = C.c_int(-1)
        from . import _native as N
        self.N, self.lib = N, N.gpu_lib()
        N.check(self.lib.fb_ctx_device(capture.ctx, C.byref(cdev)))
        self.gpu = torch.device("cuda", cdev.value)
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)

    def process(self, frames, offsets, shard_first, global_n, ts=None, timing=None):
        """One global batch: this rank's shard (host arrays `frames` / `offsets`, the frames
        [shard_first, shard_first + n) of a global batch of `global_n` frames; ts: the shard's capture
        times on a timed capture).  Every rank must call it for every global batch (an empty shard
        too).  Returns this rank's batch stats (its parse's PACKET_STATS) as a dict."""
        import time
        import torch
        N, lib, gpu = self.N, self.lib, self.gpu
        t0 = time.perf_counter()
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = offsets.size - 1
        ctx = self.cap.ctx
        d_fr = torch.from_numpy(frames if frames.size else np.zeros(1, np.uint8)).to(gpu)
        d_of = torch.from_numpy(offsets.view(np.int32)).to(gpu)
        recs = torch.empty((max(n, 1), 7), dtype=torch.int64, device=gpu)      # fb_pkt_out, 56 B
        grouped = torch.empty_like(recs)
        st = torch.zeros(N.STATS_DTYPE.itemsize // 8, dtype=torch.int64, device=gpu)
        counts = torch.zeros(self.world, dtype=torch.int64, device=gpu)
        timed = bool(getattr(self.cap, "timed", False))
        if timed:
            if ts is None or len(ts) < n:
                raise ValueError("a timed capture needs the shard's capture times")
            d_ts = torch.from_numpy(np.ascontiguousarray(ts, dtype=np.uint64).view(np.int64)).to(gpu) if n else \
                torch.zeros(1, dtype=torch.int64, device=gpu)
            ts_out = torch.empty(max(n, 1), dtype=torch.int64, device=gpu)
        torch.cuda.current_stream(gpu).synchronize()
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        N.check(lib.fb_parse_classify_dev(ctx, p(d_fr), frames.nbytes, p(d_of), n, p(recs), None, None, p(st), None))
        N.check(lib.fb_route_records_dev(ctx, p(recs), p(st), n, self.world, int(shard_first),
                                         p(d_ts) if timed else None, p(grouped), p(ts_out) if timed else None,
                                         p(counts), None))
        N.check(lib.fb_stream_sync(None))
        stats = np.frombuffer(st.cpu().numpy().tobytes(), dtype=N.STATS_DTYPE)
        cnt = [int(x) for x in counts.tolist()]
        m = sum(cnt)
        t0 = _mark(timing, gpu, "route_ms", t0)
        # all_to_all of the groups (and their capture times)
        dev = self.dev
        send = grouped[:m].to(dev)
        if self.world > 1:
            send_n = torch.tensor(cnt, dtype=torch.int64, device=dev)
            recv_n = torch.empty_like(send_n)
            self.dist.all_to_all_single(recv_n, send_n, group=self.group)
            rn = [int(x) for x in recv_n.tolist()]
            recv = torch.empty((sum(rn), 7), dtype=torch.int64, device=dev)
            self.dist.all_to_all_single(recv, send, output_split_sizes=rn, input_split_sizes=cnt, group=self.group)
            if timed:
                rts = torch.empty(sum(rn), dtype=torch.int64, device=dev)
                self.dist.all_to_all_single(rts, ts_out[:m].to(dev), output_split_sizes=rn, input_split_sizes=cnt,
                                            group=self.group)
        else:
            recv = send
            rts = ts_out[:m].to(dev) if timed else None
        t0 = _mark(timing, dev if dev.type == "cuda" else gpu, "a2a_ms", t0)
        # the owner's update: one call per global batch, its flows' packets in global order
        k = int(recv.shape[0])
        r_gpu = recv.to(gpu).contiguous() if k else torch.zeros((1, 7), dtype=torch.int64, device=gpu)
        ust = torch.zeros(N.STATS_DTYPE.itemsize // 8, dtype=torch.int64, device=gpu)
        ust[list(N.STATS_DTYPE.names).index("n_session")] = k  # (every stats field is a u64)
        keep = None
        if timed:
            g_ts = torch.zeros(max(int(global_n), 1), dtype=torch.int64, device=gpu)
            if k:
                idx = (r_gpu[:, 6] >> 32) & 0xFFFFFFFF  # pkt_index: bytes 52..55 = the high half of word 6
                g_ts[idx] = rts.to(gpu)
            keep = g_ts
        torch.cuda.current_stream(gpu).synchronize()
        if timed:
            N.check(lib.fb_set_frame_times(ctx, p(keep)))
        N.check(lib.fb_flow_update_records_dev(ctx, p(r_gpu), k, p(ust), None))
        N.check(lib.fb_stream_sync(None))
        out = np.frombuffer(ust.cpu().numpy().tobytes(), dtype=N.STATS_DTYPE)
        if int(out[0]["error"]):
            raise N.FbError(N.FB_ERR_TABLE_FULL if int(out[0]["error"]) & 4 else N.FB_ERR_INTERNAL,
                            "owner update error word %d" % int(out[0]["error"]))
        _mark(timing, gpu, "update_ms", t0)
        if timing is not None:
            timing["records_out"] = timing.get("records_out", 0) + m - cnt[self.rank]
        res = {k2: int(stats[0][k2]) for k2 in N.STATS_FIELDS if not k2.startswith("reserved")}
        res["owner_new_sessions"] = int(out[0]["new_sessions"])
        res["owner_records"] = k
        return res

    def global_table(self, with_times=False):
        """Every owner's flows (fb_flow_rec; and with_times, fb_flow_time joined by slot), gathered on
        every rank: owners in rank order."""
        import torch
        recs = self.cap.export_flows()
        rows = [np.ascontiguousarray(recs).view(np.int64).reshape(len(recs), REC_WORDS)]
        if with_times:
            t = self.cap.export_times()
            by = {int(x["slot"]): x for x in t}
            tt = np.array([by[int(r["slot"])] for r in recs], dtype=self.N.FLOW_TIME_DTYPE) if len(recs) else \
                np.zeros(0, dtype=self.N.FLOW_TIME_DTYPE)
            rows.append(np.ascontiguousarray(tt).view(np.int64).reshape(len(tt), 8))
        mine = torch.from_numpy(np.ascontiguousarray(np.concatenate(rows, axis=1) if len(rows) > 1 else rows[0]))
        width = mine.shape[1]
        if self.world == 1:
            allr = mine
        else:  # (on the group's device: RCCL takes device tensors, gloo host ones)
            mine = mine.to(self.dev)
            n = torch.tensor([mine.shape[0]], dtype=torch.int64, device=self.dev)
            sizes = [torch.zeros_like(n) for _ in range(self.world)]
            self.dist.all_gather(sizes, n, group=self.group)
            sizes = [int(x.item()) for x in sizes]
            pad = torch.zeros((max(sizes + [1]), width), dtype=torch.int64, device=self.dev)
            pad[: mine.shape[0]] = mine
            got = [torch.zeros_like(pad) for _ in range(self.world)]
            self.dist.all_gather(got, pad, group=self.group)
            allr = torch.cat([g[:sz] for g, sz in zip(got, sizes)]).cpu()
        a = allr.numpy()
        flows = np.ascontiguousarray(a[:, :REC_WORDS]).view(FLOW_REC_DTYPE).reshape(-1)
        if not with_times:
            return flows
        return flows, np.ascontiguousarray(a[:, REC_WORDS:]).view(self.N.FLOW_TIME_DTYPE).reshape(-1)
