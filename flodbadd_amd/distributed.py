"""Multi-GPU data path: packet-index shards, and the optional global per-flow counter reduce.

SURVEY.md 8e.  Decode/classify has no cross-packet state, so a batch of N*W frames shards by
contiguous packet-index range: rank r owns [r*N, (r+1)*N) and runs its own context with no
data-path collective (bench.py reports "scaling": "weak").  The one real exchange is the global
per-flow count (BASELINE config C5):
  1. every rank exports its flow table (canonical key + 6 integer counters, fb_flow_export);
  2. all-gather of the keys (keys << packets);
  3. every rank sorts the union by the derived Ord of Session (src/sessions.rs:23-30: protocol,
     src_ip [V4 < V6, then octets], src_port, dst_ip, dst_port) -> an identical dense flow_id;
  4. each rank scatters its counters into a dense int64[F][6];
  5. all_reduce(SUM) -- over RCCL/xGMI with device tensors ("nccl" backend), gloo on the CPU.
Integer sums are order independent, so the result is bit-identical to a single-GPU table.
The ordered per-flow state merges the same way once positions are made global (rank r's
pkt_index + its shard's first index): first_seen = MIN, last_seen = MAX, end_seen = MIN (the
earliest FIN/RST), hist_len = SUM, hist_mask = OR (a SUM of per-bit 4-bit fields, since RCCL has
no bitwise reduction).  conn_state is re-decided from the ending rank's end_mask OR the characters
of the ranks before it -- exact when every rank's table holds one update call of the same global
batch (C5), since the earlier ranks' packets then all precede the end packet.
"""
import numpy as np

from ._native import FB_SEEN_NONE, FLOW_REC_DTYPE

COUNTERS = ("outbound_bytes", "inbound_bytes", "orig_pkts", "resp_pkts", "orig_ip_bytes", "resp_ip_bytes")


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
    """Row order of [F,10] key words by the derived Ord of Session."""
    src, dst = words[:, 0:4], words[:, 4:8]
    ports, pf = words[:, 8], words[:, 9]
    sport, dport = ports & 0xFFFF, ports >> 16
    proto, fam = pf & 0xFF, (pf >> 8) & 0xFF
    cols = [dport, dst[:, 3], dst[:, 2], dst[:, 1], dst[:, 0], sport, src[:, 3], src[:, 2], src[:, 1], src[:, 0],
            fam, proto]
    return np.lexsort(cols)  # last column is the primary key


def _conn_state(m):
    """determine_conn_state (src/packets.rs:539-559) over FB_HIST_CHARS bits (vectorised)."""
    b = lambda k: (m >> k) & 1 == 1
    S, H, h, F, f, R, r = b(0), b(2), b(3), b(4), b(5), b(6), b(7)
    return np.select([S & H & F & f, S & ~h & ~r, R | r, S & H & ~F & ~f], [1, 2, 3, 4], 5).astype(np.uint8)


def global_flow_table(dist, flows, device=None, group=None, shard_first=0):
    """All ranks' flow tables merged into one table sorted by Session's derived Ord, identical
    on every rank.  `dist` is torch.distributed (initialised); `device` is the torch device of
    the collective tensors (a cuda device for RCCL, None/cpu for gloo); `shard_first` is the
    global index of this rank's first packet (shard_range)."""
    import torch
    flows = np.ascontiguousarray(flows, dtype=FLOW_REC_DTYPE)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert world < 16, "hist_mask OR uses 4-bit fields"
    kw = _key_words(flows).astype(np.int64)  # u32 words widened (exact)
    n = torch.tensor([len(flows)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes + [1])
    pad = torch.zeros((m, 10), dtype=torch.int64, device=device)
    if len(flows):
        pad[: len(flows)] = torch.from_numpy(kw).to(device)
    gathered = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad, group=group)
    allk = np.concatenate([g[:s].cpu().numpy() for g, s in zip(gathered, sizes)]).astype(np.uint32)
    # unique keys, dense ids in derived-Ord order
    uniq = np.unique(allk.view(np.dtype((np.void, 40))).ravel()).view(np.uint32).reshape(-1, 10)
    order = sort_keys(uniq)
    uniq = uniq[order]
    F = len(uniq)
    ukey = uniq.view(np.dtype((np.void, 40))).ravel()
    mine = _key_words(flows).view(np.dtype((np.void, 40))).ravel()
    # position of each local key in the (void-sorted) unique array, then in the Ord order
    vsort = np.argsort(ukey)
    idx = vsort[np.searchsorted(ukey[vsort], mine)] if len(flows) else np.zeros(0, dtype=np.int64)

    def reduce(cols, fill, op):
        a = np.full((F, len(cols)), fill, dtype=np.int64)
        if len(flows):
            a[idx] = np.stack(cols, axis=1)
        t = torch.from_numpy(a).to(device)
        dist.all_reduce(t, op=op, group=group)
        return t.cpu().numpy()

    def glob(pos):  # rank-local position -> global ((call << 32) | global packet index)
        pos = pos.astype(np.uint64)
        return ((pos >> np.uint64(32)) << np.uint64(32)) | ((pos & np.uint64(0xFFFFFFFF)) + np.uint64(shard_first))

    big = np.iinfo(np.int64).max
    mask = flows["hist_mask"].astype(np.int64)
    spread = np.zeros(len(flows), dtype=np.int64)
    for b in range(13):
        spread |= ((mask >> b) & 1) << (4 * b)
    ended = flows["end_seen"] != np.uint64(FB_SEEN_NONE)
    end = np.where(ended, glob(flows["end_seen"]).astype(np.int64), big)
    sums = reduce([flows[c].astype(np.int64) for c in COUNTERS] + [flows["hist_len"].astype(np.int64), spread],
                  0, dist.ReduceOp.SUM)
    mins = reduce([glob(flows["first_seen"]).astype(np.int64), end], big, dist.ReduceOp.MIN)
    last = reduce([glob(flows["last_seen"]).astype(np.int64)], -1, dist.ReduceOp.MAX)
    # conn_state: the ending rank's end_mask | the conn_state characters of the ranks before it
    gend = mins[:, 1]
    my_end = np.full(F, big, dtype=np.int64)
    my_end[idx] = end
    is_end_rank = (my_end == gend) & (gend != big)
    end_rank = reduce([np.where(is_end_rank[idx], rank, 0)], 0, dist.ReduceOp.SUM)[:, 0]
    # ranks before the ending one add their S s H h F f R r bits, the ending rank its end_mask
    before = np.where(rank < end_rank[idx], mask & 0xFF, 0) | \
        np.where(is_end_rank[idx], flows["end_mask"].astype(np.int64), 0)
    bits = np.zeros(len(flows), dtype=np.int64)
    for b in range(8):
        bits |= ((before >> b) & 1) << (4 * b)
    emask_sum = reduce([bits], 0, dist.ReduceOp.SUM)[:, 0]
    emask = np.zeros(F, dtype=np.int64)
    hmask = np.zeros(F, dtype=np.int64)
    for b in range(13):
        hmask |= (((sums[:, 7] >> (4 * b)) & 15) > 0).astype(np.int64) << b
        if b < 8:
            emask |= (((emask_sum >> (4 * b)) & 15) > 0).astype(np.int64) << b

    out = np.zeros(F, dtype=FLOW_REC_DTYPE)
    out.view(np.uint8).reshape(F, FLOW_REC_DTYPE.itemsize)[:, :40] = uniq.view(np.uint8).reshape(F, 40)
    for j, c in enumerate(COUNTERS):
        out[c] = sums[:, j].astype(np.uint64)
    has_end = gend != big
    out["hist_len"] = sums[:, 6].astype(np.uint32)
    out["hist_mask"] = hmask.astype(np.uint16)
    out["first_seen"] = mins[:, 0].astype(np.uint64)
    out["last_seen"] = last[:, 0].astype(np.uint64)
    out["end_seen"] = np.where(has_end, gend.astype(np.uint64), np.uint64(FB_SEEN_NONE))
    out["end_mask"] = np.where(has_end, emask, 0).astype(np.uint8)
    out["conn_state"] = np.where(has_end, _conn_state(emask), 0).astype(np.uint8)
    return out
