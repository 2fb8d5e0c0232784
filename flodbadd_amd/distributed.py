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


def global_flow_table(dist, flows, device=None, group=None):
    """All ranks' flow tables merged into one table sorted by Session's derived Ord, identical
    on every rank.  `dist` is torch.distributed (initialised); `device` is the torch device of
    the collective tensors (a cuda device for RCCL, None/cpu for gloo)."""
    import torch
    flows = np.ascontiguousarray(flows, dtype=FLOW_REC_DTYPE)
    world = dist.get_world_size(group)
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
    dense = np.zeros((F, 6), dtype=np.int64)
    if len(flows):
        dense[idx] = np.stack([flows[c].astype(np.int64) for c in COUNTERS], axis=1)
    t = torch.from_numpy(dense).to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    dense = t.cpu().numpy()
    out = np.zeros(F, dtype=FLOW_REC_DTYPE)
    out.view(np.uint8).reshape(F, FLOW_REC_DTYPE.itemsize)[:, :40] = uniq.view(np.uint8).reshape(F, 40)
    for j, c in enumerate(COUNTERS):
        out[c] = dense[:, j].astype(np.uint64)
    return out
