"""Multi-GPU data path: packet-index shards, and the optional global per-flow counter reduce.

SURVEY.md 8e.  Decode/classify has no cross-packet state, so a batch of N*W frames shards by
contiguous packet-index range: rank r owns [r*N, (r+1)*N) and runs its own context with no
data-path collective (bench.py reports "scaling": "weak").  The one real exchange is the global
per-flow count (BASELINE config C5):
  1. every rank exports its flow table (canonical key + 6 integer counters, fb_flow_export);
  2. all-gather of the keys (keys << packets);
  3. every rank sorts the union by the derived Ord of Session (src/sessions.rs:23-30: protocol,
     src_ip [V4 < V6, then octets], src_port, dst_ip, dst_port) -> an identical dense flow_id
     (an LSD sort of the keys' Ord columns on the collective's device);
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

from ._native import FLOW_REC_DTYPE

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
    """determine_conn_state (src/packets.rs:539-559) over FB_HIST_CHARS bits (vectorised, torch)."""
    import torch
    b = lambda k: ((m >> k) & 1) == 1
    S, H, h, F, f, R, r = b(0), b(2), b(3), b(4), b(5), b(6), b(7)
    c = torch.full_like(m, 5)
    c = torch.where(S & H & ~F & ~f, torch.full_like(m, 4), c)
    c = torch.where(R | r, torch.full_like(m, 3), c)
    c = torch.where(S & ~h & ~r, torch.full_like(m, 2), c)
    return torch.where(S & H & F & f, torch.full_like(m, 1), c)  # np.select order: first match wins


def _hi32(x):
    """x (int64 holding a u32) << 32 without leaving int64: sign-extend bit 31 first."""
    return ((x ^ 0x80000000) - 0x80000000) << 32


def _ord_sort(cols):
    """Permutation sorting the rows of [T,12] int64 Ord columns lexicographically (column 0
    primary): one stable sort per column, least significant first (LSD), all on cols' device."""
    import torch
    perm = torch.arange(cols.shape[0], device=cols.device)
    for c in range(cols.shape[1] - 1, -1, -1):
        _, o = torch.sort(cols[perm, c], stable=True)
        perm = perm[o]
    return perm


def global_flow_table(dist, flows, device=None, group=None, shard_first=0):
    """All ranks' flow tables merged into one table sorted by Session's derived Ord, identical
    on every rank.  `dist` is torch.distributed (initialised); `device` is the torch device of
    the collective tensors (a cuda device for RCCL, None/cpu for gloo); `shard_first` is the
    global index of this rank's first packet (shard_range).  Everything between the upload of
    the exported records and the download of the merged columns runs as torch ops on `device`:
    the keys' Ord columns, their all-gather, an LSD sort of the union, dense ids from adjacent
    differences, the scatters and the all-reduces."""
    import torch
    dev = torch.device("cpu") if device is None else torch.device(device)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert world < 16, "hist_mask OR uses 4-bit fields"
    if isinstance(flows, torch.Tensor):  # [n, 128] uint8 on `dev` (fb_flow_export_dev)
        raw = flows.to(dev).reshape(-1, FLOW_REC_DTYPE.itemsize)
    else:
        flows = np.ascontiguousarray(flows, dtype=FLOW_REC_DTYPE)
        raw = torch.from_numpy(flows.view(np.uint8).reshape(len(flows), FLOW_REC_DTYPE.itemsize)).to(dev)
    nl = int(raw.shape[0])
    w32 = raw.view(torch.int32).to(torch.int64) & 0xFFFFFFFF  # [nl, 32] u32 words, widened
    w64 = raw.view(torch.int64)                                # [nl, 16] u64 words (as int64 bits)
    ports, pf = w32[:, 8], w32[:, 9]
    # key columns in the derived Ord's priority: protocol, family (V4 < V6), src words, src port,
    # dst words, dst port (src/sessions.rs:23-30; IpAddr octets big-endian = the words' order)
    mine = torch.stack([pf & 0xFF, (pf >> 8) & 0xFF, w32[:, 0], w32[:, 1], w32[:, 2], w32[:, 3], ports & 0xFFFF,
                        w32[:, 4], w32[:, 5], w32[:, 6], w32[:, 7], ports >> 16], dim=1)
    n = torch.tensor([nl], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes + [1])
    pad = torch.zeros((m, 12), dtype=torch.int64, device=dev)
    pad[:nl] = mine
    gathered = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad, group=group)
    allc = torch.cat([g[:sz] for g, sz in zip(gathered, sizes)])
    # dense ids in Ord order: sort the union, a new id wherever a row differs from the one before
    perm = _ord_sort(allc)
    srt = allc[perm]
    first = torch.ones(srt.shape[0], dtype=torch.bool, device=dev)
    if srt.shape[0] > 1:
        first[1:] = (srt[1:] != srt[:-1]).any(dim=1)
    ids = torch.cumsum(first.to(torch.int64), 0) - 1
    inv = torch.empty_like(ids)
    inv[perm] = ids
    uniq = srt[first]
    F = int(uniq.shape[0])
    start = sum(sizes[:rank])
    idx = inv[start:start + nl]

    def reduce(cols, fill, op):
        t = torch.full((F, len(cols)), fill, dtype=torch.int64, device=dev)
        if nl:
            t[idx] = torch.stack(cols, dim=1)
        dist.all_reduce(t, op=op, group=group)
        return t

    def glob(pos):  # rank-local position -> global ((call << 32) | global packet index)
        return ((pos >> 32) << 32) | ((pos & 0xFFFFFFFF) + shard_first)

    big = torch.iinfo(torch.int64).max
    counters, first_seen, last_seen, end_seen = w64[:, 5:11], w64[:, 11], w64[:, 12], w64[:, 13]
    hist_len, state = w32[:, 28], w32[:, 29]
    mask, end_mask = state & 0xFFFF, (state >> 24) & 0xFF
    spread = torch.zeros(nl, dtype=torch.int64, device=dev)
    for b in range(13):
        spread |= ((mask >> b) & 1) << (4 * b)
    ended = end_seen != -1  # FB_SEEN_NONE
    end = torch.where(ended, glob(end_seen), torch.full_like(end_seen, big))
    sums = reduce([counters[:, j] for j in range(6)] + [hist_len, spread], 0, dist.ReduceOp.SUM)
    mins = reduce([glob(first_seen), end], big, dist.ReduceOp.MIN)
    # session_flags (stored at insert) are a function of the key and the configuration, the same on
    # every rank that holds the flow: MAX keeps them
    last = reduce([glob(last_seen), w32[:, 31]], -1, dist.ReduceOp.MAX)
    # conn_state: the ending rank's end_mask | the conn_state characters of the ranks before it
    gend = mins[:, 1]
    is_end = (end == gend[idx]) & (gend[idx] != big)
    end_rank = reduce([torch.where(is_end, rank, 0)], 0, dist.ReduceOp.SUM)[:, 0]
    # ranks before the ending one add their S s H h F f R r bits, the ending rank its end_mask
    before = torch.where(rank < end_rank[idx], mask & 0xFF, 0) | torch.where(is_end, end_mask, 0)
    bits = torch.zeros(nl, dtype=torch.int64, device=dev)
    for b in range(8):
        bits |= ((before >> b) & 1) << (4 * b)
    emask_sum = reduce([bits], 0, dist.ReduceOp.SUM)[:, 0]
    hmask = torch.zeros(F, dtype=torch.int64, device=dev)
    emask = torch.zeros(F, dtype=torch.int64, device=dev)
    for b in range(13):
        hmask |= (((sums[:, 7] >> (4 * b)) & 15) > 0).to(torch.int64) << b
        if b < 8:
            emask |= (((emask_sum >> (4 * b)) & 15) > 0).to(torch.int64) << b

    # the merged records assembled as fb_flow_rec words on the device, one download
    has_end = gend != big
    w = torch.zeros((F, 16), dtype=torch.int64, device=dev)
    kw = [uniq[:, 2], uniq[:, 3], uniq[:, 4], uniq[:, 5], uniq[:, 7], uniq[:, 8], uniq[:, 9], uniq[:, 10],
          uniq[:, 6] | (uniq[:, 11] << 16), uniq[:, 0] | (uniq[:, 1] << 8)]
    for j in range(5):
        w[:, j] = kw[2 * j] | _hi32(kw[2 * j + 1])
    w[:, 5:11] = sums[:, 0:6]
    w[:, 11] = mins[:, 0]
    w[:, 12] = last[:, 0]
    w[:, 13] = torch.where(has_end, gend, torch.full_like(gend, -1))  # FB_SEEN_NONE
    em = torch.where(has_end, emask, 0)
    cs = torch.where(has_end, _conn_state(emask), 0)
    w[:, 14] = sums[:, 6] | _hi32(hmask | (cs << 16) | (em << 24))
    w[:, 15] = _hi32(last[:, 1])  # slot 0, session_flags
    return w.cpu().numpy().view(FLOW_REC_DTYPE).reshape(F)
