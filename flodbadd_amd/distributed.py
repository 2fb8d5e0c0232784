"""Multi-GPU data path: packet-index shards, and the optional global per-flow merge.

SURVEY.md 8e.  Decode/classify has no cross-packet state, so a batch of N*W frames shards by
contiguous packet-index range: rank r owns [r*N, (r+1)*N) and runs its own context with no
data-path collective (bench.py reports "scaling": "weak").  The one real exchange is the global
per-flow table (BASELINE config C5), O(F) per rank:
  1. every rank exports its flow table (fb_flow_export[_dev]: canonical key, 6 integer counters,
     ordered state) and makes its positions global (+ its shard's first packet index);
  2. owner ranks by ranges of Session's derived Ord (src/sessions.rs:23-30: protocol, src_ip
     [V4 < V6, then octets], src_port, dst_ip, dst_port): W-1 splitters from an all-gathered
     sample of keys, the same on every rank;
  3. all_to_all of the 128-B records to their owners (RCCL over xGMI with device tensors, gloo on
     the CPU);
  4. each owner sorts what it received by Ord (the key's non-constant fields packed into 63-bit
     words, one stable sort per word) and merges equal keys: integer sums, MIN first_seen and
     end_seen, MAX last_seen, hist_len = SUM, hist_mask = OR (a SUM of per-bit 4-bit fields,
     no rank holds a key twice), conn_state re-decided from the ending rank's end_mask OR the
     characters of the ranks before it -- exact when every rank's table holds one update call of
     the same global batch (C5), since the earlier ranks' packets then all precede the end packet;
  5. all-gather of the merged records: owner ranges are Ord ranges, so rank order IS Ord order.
Bytes per rank: ~128 B x its flows out (x (W-1)/W) and in, and 128 B x the global flows gathered.
Integer sums are order independent, so the result is bit-identical to a single-GPU table.
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


_LUTS = {}


def _luts(device):
    """Lookup tables for the hist_mask OR-as-SUM: 8 bits -> 4-bit fields, and 4 nibble-flags
    (bits 0, 4, 8, 12 of a 16-bit chunk) -> 4 bits."""
    import torch
    key = str(device)
    if key not in _LUTS:
        v = np.arange(256, dtype=np.int64)
        spread = np.zeros(256, dtype=np.int64)
        for b in range(8):
            spread |= ((v >> b) & 1) << (4 * b)
        c = np.arange(1 << 16, dtype=np.int64)
        pack = ((c >> 0) & 1) | (((c >> 4) & 1) << 1) | (((c >> 8) & 1) << 2) | (((c >> 12) & 1) << 3)
        _LUTS[key] = (torch.from_numpy(spread).to(device), torch.from_numpy(pack).to(device))
    return _LUTS[key]


def _spread(mask, device):
    """Bit b of a 16-bit mask -> bit 4 b (so a SUM over < 16 rows is an OR per bit)."""
    spread, _ = _luts(device)
    return spread[mask & 0xFF] | (spread[(mask >> 8) & 0xFF] << 32)


def _unspread(x, nbits, device):
    """Bit b set <=> 4-bit field b of x is non-zero (b < nbits)."""
    _, pack = _luts(device)
    t = x | (x >> 1) | (x >> 2) | (x >> 3)
    t = t & 0x1111111111111111
    out = pack[t & 0xFFFF] | (pack[(t >> 16) & 0xFFFF] << 4) | (pack[(t >> 32) & 0xFFFF] << 8) | \
        (pack[(t >> 48) & 0xFFFF] << 12)
    return out & ((1 << nbits) - 1)


def _hi32(x):
    """x (int64 holding a u32) << 32 without leaving int64: sign-extend bit 31 first."""
    return ((x ^ 0x80000000) - 0x80000000) << 32


def _ord_fields(rows):
    """The key's Ord fields (value, bits) of [n, 16] int64 flow records, in priority order:
    protocol, family (V4 < V6), src words, src port, dst words, dst port (IpAddr octets big-endian =
    the words' order)."""
    import torch
    w = rows.view(torch.int32)

    def u32(j):
        return w[:, j].to(torch.int64) & 0xFFFFFFFF

    ports, pf = u32(8), u32(9)
    return [(pf & 0xFF, 8), ((pf >> 8) & 0xFF, 8), (u32(0), 32), (u32(1), 32), (u32(2), 32), (u32(3), 32),
            (ports & 0xFFFF, 16), (u32(4), 32), (u32(5), 32), (u32(6), 32), (u32(7), 32), (ports >> 16, 16)]


_FIELD_WORD = (9, 9, 0, 1, 2, 3, 8, 4, 5, 6, 7, 8)  # the key word each Ord field comes from


def _pack63(fields, rows=None):
    """The fields' bits, most significant first, in 63-bit words (non-negative int64): comparing
    the word lists lexicographically compares the fields.  With `rows` ([n, 16] int64 records),
    fields whose key word is equal on every row are left out (they cannot order those rows):
    one comparison over the ten key words, one host sync."""
    import torch
    if rows is not None and rows.shape[0] > 1:
        kw = rows.view(torch.int32)[:, :10]
        varies = (kw != kw[:1]).any(dim=0).tolist()
        fields = [f for f, j in zip(fields, _FIELD_WORD) if varies[j]]
    words, cur, used = [], None, 0
    for v, bits in fields:
        while bits > 0:
            take = min(bits, 63 - used)
            part = (v >> (bits - take)) & ((1 << take) - 1)
            cur = part if cur is None else (cur << take) | part
            used += take
            bits -= take
            v = v & ((1 << bits) - 1)
            if used == 63:
                words.append(cur)
                cur, used = None, 0
    if cur is not None:
        words.append(cur << (63 - used))
    return words


def _lsd_order(words, n, device):
    """Permutation sorting rows by the word list (word 0 most significant): one stable sort per
    word, least significant first."""
    import torch
    perm = torch.arange(n, device=device)
    for wd in reversed(words):
        _, o = torch.sort(wd[perm], stable=True)
        perm = perm[o]
    return perm


def _owners(dist, group, world, words, n, device, sample=1024):
    """Owner rank of each row: the number of the W-1 Ord splitters at or below its key.  The
    splitters are quantiles of an all-gathered sample (up to `sample` rows per rank), sorted the
    same way on every rank."""
    import torch
    k = len(words)
    take = min(n, sample)
    idx = (torch.arange(take, device=device) * n) // max(take, 1)
    mine = torch.zeros((sample, k), dtype=torch.int64, device=device)
    if take:
        mine[:take] = torch.stack([wd[idx] for wd in words], dim=1)
    cnt = torch.tensor([take], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    got = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(got, mine, group=group)
    smp = torch.cat([g[:int(c.item())] for g, c in zip(got, cnts)]).cpu().numpy()
    order = np.lexsort([smp[:, j] for j in range(k - 1, -1, -1)]) if len(smp) else np.zeros(0, np.int64)
    spl = smp[order[[(j * len(order)) // world for j in range(1, world)]]] if len(smp) else np.zeros((0, k), np.int64)
    owner = torch.zeros(n, dtype=torch.int64, device=device)
    for s in spl:  # owner += (row >= splitter), lexicographic over the words
        lt = torch.zeros(n, dtype=torch.bool, device=device)
        for j in range(k - 1, -1, -1):
            lt = (words[j] < int(s[j])) | ((words[j] == int(s[j])) & lt)
        owner += (~lt).to(torch.int64)
    return owner


def global_flow_table(dist, flows, device=None, group=None, shard_first=0, as_tensor=False):
    """All ranks' flow tables merged into one table sorted by Session's derived Ord, identical
    on every rank.  `dist` is torch.distributed (initialised); `device` is the torch device of
    the collective tensors (a cuda device for RCCL, None/cpu for gloo); `shard_first` is the
    global index of this rank's first packet (shard_range).  Returns FLOW_REC_DTYPE records, or
    with as_tensor=True the [F, 128] uint8 tensor on `device` (no download).  Everything runs as
    torch ops on `device`: owners by Ord splitters, all_to_all of the records, the owner's sort
    and merge, the all-gather of merged records."""
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
    # [nl, 16] u64 words (as int64 bits)
    rows = raw.contiguous().view(torch.int64) if nl else torch.zeros((0, 16), dtype=torch.int64, device=dev)
    if shard_first:  # rank-local positions -> global ((call << 32) | global packet index)
        rows = rows.clone()
        for j in (11, 12, 13):
            pos = rows[:, j]
            g = ((pos >> 32) << 32) | ((pos & 0xFFFFFFFF) + shard_first)
            rows[:, j] = g if j != 13 else torch.where(pos != -1, g, pos)  # end_seen NONE stays
    # 2-3. owners by Ord range, records to their owners
    if world > 1:
        owner = _owners(dist, group, world, _pack63(_ord_fields(rows)), nl, dev)
        order = torch.sort(owner, stable=True)[1]
        send = rows[order].contiguous()
        send_n = torch.bincount(owner, minlength=world)
        recv_n = torch.empty_like(send_n)
        dist.all_to_all_single(recv_n, send_n, group=group)
        rn = recv_n.tolist()
        recv = torch.empty((sum(rn), 16), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv, send, output_split_sizes=rn, input_split_sizes=send_n.tolist(), group=group)
        src = torch.repeat_interleave(torch.arange(world, device=dev), recv_n)
    else:
        recv, src = rows, torch.zeros(nl, dtype=torch.int64, device=dev)
    m = int(recv.shape[0])
    # 4. sort by Ord, merge equal keys
    words = _pack63(_ord_fields(recv), recv)
    if m > 1 and words:
        perm = _lsd_order(words, m, dev)
        recv, src = recv[perm], src[perm]
        words = [wd[perm] for wd in words]
    first = torch.ones(m, dtype=torch.bool, device=dev)
    if m > 1:
        first[1:] = False
        for wd in words:
            first[1:] |= wd[1:] != wd[:-1]
    F = int(first.sum().item()) if m else 0
    dup = F != m
    gid = torch.cumsum(first.to(torch.int64), 0) - 1 if dup else None

    def seg(vals, op, fill):  # per merged key: op over its rows (identity when no key repeats)
        if not dup:
            return vals
        t = torch.full((F,) + tuple(vals.shape[1:]), fill, dtype=torch.int64, device=dev)
        if op == "sum":
            return t.index_add_(0, gid, vals)
        ix = gid.view(-1, *([1] * (vals.dim() - 1))).expand_as(vals)
        return t.scatter_reduce_(0, ix, vals, reduce=op, include_self=True)

    def at(x):  # a per-key value back at its rows
        return x[gid] if dup else x

    big = torch.iinfo(torch.int64).max
    w32 = recv.view(torch.int32)
    hist_len = w32[:, 28].to(torch.int64) & 0xFFFFFFFF
    state = w32[:, 29].to(torch.int64) & 0xFFFFFFFF
    flags = w32[:, 31].to(torch.int64) & 0xFFFFFFFF
    mask, end_mask = state & 0xFFFF, (state >> 24) & 0xFF
    end_seen = recv[:, 13]
    end = torch.where(end_seen != -1, end_seen, torch.full_like(end_seen, big))
    if dup:
        sums = seg(torch.cat([recv[:, 5:11], hist_len[:, None], _spread(mask, dev)[:, None]], dim=1), "sum", 0)
        mins = seg(torch.stack([recv[:, 11], end], dim=1), "amin", big)
        last = seg(torch.stack([recv[:, 12], flags], dim=1), "amax", -1)
        # conn_state: the ending rank's end_mask | the conn_state characters of the ranks before it
        gend = mins[:, 1]
        is_end = (end == at(gend)) & (at(gend) != big)
        end_rank = seg(torch.where(is_end, src, 0), "sum", 0)
        before = torch.where(src < at(end_rank), mask & 0xFF, 0) | torch.where(is_end, end_mask, 0)
        emask = _unspread(seg(_spread(before, dev), "sum", 0), 8, dev)
        hmask = _unspread(sums[:, 7], 13, dev)
    else:  # no key met twice: every reduction is the row itself (the ending row is its own)
        sums = torch.cat([recv[:, 5:11], hist_len[:, None]], dim=1)
        mins = torch.stack([recv[:, 11], end], dim=1)
        last = torch.stack([recv[:, 12], flags], dim=1)
        gend = end
        emask = torch.where(end != big, end_mask, 0)
        hmask = mask
    # the merged records as fb_flow_rec words
    has_end = gend != big
    w = torch.empty((F, 16), dtype=torch.int64, device=dev)
    w[:, 0:5] = recv[first, 0:5] if dup else recv[:, 0:5]
    w[:, 5:11] = sums[:, 0:6]
    w[:, 11] = mins[:, 0]
    w[:, 12] = last[:, 0]
    w[:, 13] = torch.where(has_end, gend, torch.full_like(gend, -1))  # FB_SEEN_NONE
    em = torch.where(has_end, emask, 0)
    cs = torch.where(has_end, _conn_state(emask), 0)
    w[:, 14] = sums[:, 6] | _hi32(hmask | (cs << 16) | (em << 24))
    w[:, 15] = _hi32(last[:, 1])  # slot 0, session_flags
    # 5. owners' ranges in rank order = Ord order
    if world > 1:
        n = torch.tensor([F], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(x.item()) for x in sizes]
        pad = torch.zeros((max(sizes + [1]), 16), dtype=torch.int64, device=dev)
        pad[:F] = w
        got = [torch.zeros_like(pad) for _ in range(world)]
        dist.all_gather(got, pad, group=group)
        w = torch.cat([g[:sz] for g, sz in zip(got, sizes)])
    out = w.view(torch.uint8).reshape(-1, FLOW_REC_DTYPE.itemsize)
    if as_tensor:
        return out
    return w.cpu().numpy().view(FLOW_REC_DTYPE).reshape(-1)
