"""CPU model (no GPU): what combining a hot flow's records INSIDE the parse would leave for K1c
under the C4 Zipf(1.1) batch.  Parses the synthetic batch with the C oracle (test infrastructure,
used here only to get each SESSION record's flow), then counts, for a combining window of W
consecutive frames (64 = one wavefront's segment, 256 / 1024 / 4096 = a parse workgroup's or a
larger staging window), the records left and K1's hot (chunk, partition) groups -- groups of >= 64
records in a 20,480-record chunk (kCombMin, FB_FLOW_CHUNK; 4,096 partitions at the bench's 2^21
table) -- that K1c would still reduce.  Partition = a fixed random function of the flow (the
distribution, not fb_flow_hash's exact bits, is what matters here).  Prints a markdown table."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10 * (1 << 20)
    from flodbadd_amd import synth
    from oracle import coracle
    fr, of = synth.generate(4, n, zipf=1, zipf_s=1.1)
    recs, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), fr, of)
    a = np.concatenate([recs["src_ip"], recs["src_port"][:, None].astype(np.uint32)], axis=1)
    b = np.concatenate([recs["dst_ip"], recs["dst_port"][:, None].astype(np.uint32)], axis=1)
    swap = np.lexsort(np.concatenate([a, b], axis=1).T[::-1])  # (not needed: canonical pair below)
    del swap
    less = np.zeros(len(recs), dtype=bool)
    eq = np.ones(len(recs), dtype=bool)
    for c in range(5):
        less |= eq & (a[:, c] < b[:, c])
        eq &= a[:, c] == b[:, c]
    lo = np.where(less[:, None], a, b)
    hi = np.where(less[:, None], b, a)
    key = np.concatenate([lo, hi, recs["protocol"][:, None].astype(np.uint32)], axis=1)
    _, flow = np.unique(key, axis=0, return_inverse=True)
    flow = flow.ravel().astype(np.int64)
    pkt = recs["pkt_index"].astype(np.int64)
    parts = 4096
    rng = np.random.default_rng(7)
    part_of = rng.integers(0, parts, size=flow.max() + 1)
    chunk_recs = 20480

    def k1c_load(sel_flow):
        """hot groups and their records for records (in order) of the given flows"""
        m = len(sel_flow)
        ch = np.arange(m) // chunk_recs
        g = ch * parts + part_of[sel_flow]
        cnt = np.bincount(g)
        hot = cnt >= 64
        return int(hot.sum()), int(cnt[hot].sum())

    rows = []
    hg, hr = k1c_load(flow)
    rows.append(("none (product)", len(flow), hg, hr))
    for w in (64, 256, 1024, 4096, 20480):
        win = pkt // w
        # one record per (window, flow), in first-occurrence order
        comb = win * (flow.max() + 1) + flow
        _, first = np.unique(comb, return_index=True)
        keep = np.sort(first)
        hg, hr = k1c_load(flow[keep])
        rows.append(("%d frames" % w, len(keep), hg, hr))
    print("C4 Zipf(1.1), %d frames, %d SESSION records, %d flows" % (n, len(flow), flow.max() + 1))
    print("| combining window | records to K1 | K1c hot groups | records in hot groups |")
    print("|---|---|---|---|")
    for r in rows:
        print("| %s | %d | %d | %d |" % r)


if __name__ == "__main__":
    main()
