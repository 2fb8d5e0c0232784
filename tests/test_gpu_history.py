"""GPU ordered per-flow state against the oracle, bit-exact.

The flow table's ordered fields -- first / last / end positions (start_time, last_activity,
end_time stand-ins), hist_len, hist_mask, conn_state, end_mask -- must equal the oracle's rows,
and the history strings rebuilt from fb_flow_history_dev batch by batch must equal the oracle's
`history` (src/packets.rs:187-198, 410-426; map_tcp_flags 561-601; determine_conn_state 539-559).
"""
import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from flodbadd_amd.capture import FlodbaddGpuCapture
from flodbadd_amd.sessions import SessionFilter
from oracle import coracle
from test_gpu_parity import rows_sorted

pytestmark = pytest.mark.gpu


def _check_tables(cap, flows):
    gf = cap.export_flows()
    rf = flows.export_sorted()
    assert len(gf) == len(rf)
    assert rows_sorted(gf) == rows_sorted(rf)
    for r in gf:
        h, cs = flows.history(r)
        assert cap.histories.get(int(r["slot"]), "") == h, (r, h)
        assert N.CONN_STATES[int(r["conn_state"])] == cs
        assert int(r["hist_len"]) == len(h)
    return gf


def _run(batches, seg=False, capacity=1 << 20):
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=capacity, track_history=True)
    flows = coracle.Flows()
    cfg = coracle.make_cfg(2)
    try:
        for frames, offs in batches:
            g = cap.process_frames_seg(frames, offs) if seg else cap.process_frames(frames, offs)
            r_out, _, _, _ = coracle.parse_classify(cfg, frames, offs)
            assert g.records.tobytes() == r_out.tobytes()
            flows.update(r_out)
        return _check_tables(cap, flows)
    finally:
        cap.close()


@pytest.mark.parametrize("seg", [False, True], ids=["dense", "seg"])
def test_history_synthetic_zipf(seg):
    """Three Zipf(1.1) batches (hot flows with thousands of packets spanning batches)."""
    batches = [synth.generate(4, 150000, first=b * 150000, zipf=1, zipf_s=1.1) for b in range(3)]
    gf = _run(batches, seg=seg)
    assert (gf["hist_len"] > 100).any() and (gf["conn_state"] > 0).any()


def test_history_zipf_split_partitions():
    """Batches of more than 16 bucketing chunks with Zipf(1.1) popularity: the hottest flows' partitions
    carry tens of thousands of characters, so the history splits them over chunk blocks (per-block
    slot counts first, k_hist_general<true>); every flow's history string equals the oracle's."""
    batches = [synth.generate(4, 700000, first=0, zipf=1, zipf_s=1.1),
               synth.generate(4, 400000, first=700000, zipf=1, zipf_s=1.1)]
    gf = _run(batches, seg=True)
    assert (gf["hist_len"] > 40000).any()


def _flow(src, sport, dst, dport):
    out = lambda fl, n=0: fg.tcp_frame(src, sport, dst, dport, fl, n)
    back = lambda fl, n=0: fg.tcp_frame(dst, dport, src, sport, fl, n)
    return out, back


def hand_batches():
    """Hand-built flows through the conn_state outcomes, ends in earlier/later batches, an empty
    batch in between, a UDP flow (no history) and flows interleaved inside each batch."""
    a_o, a_b = _flow("10.0.0.1", 40001, "1.1.1.1", 443)   # S h A > < | F f
    b_o, b_b = _flow("10.0.0.2", 40002, "1.1.1.2", 443)   # F first (ends there), then S ... h
    c_o, _ = _flow("10.0.0.3", 40003, "1.1.1.3", 443)     # R as the first packet
    d_o, _ = _flow("10.0.0.4", 40004, "1.1.1.4", 443)     # SYN|FIN: character S, ends the flow
    e_o, e_b = _flow("10.0.0.5", 40005, "1.1.1.5", 443)   # S | h | r A across three batches
    f_o, f_b = _flow("10.0.0.6", 40006, "1.1.1.6", 443)   # S H F in batch 1, more packets later
    g_o, g_b = _flow("10.0.0.8", 40008, "1.1.1.8", 443)   # S H > F | f: S0 (f comes after the end)
    h_o, h_b = _flow("10.0.0.9", 40009, "1.1.1.9", 443)   # S H h then SYN|RST (character S): S1
    # (SF needs both F and f at the first FIN/RST, which a FIN-only end never has)
    S, A, F, R, P = fg.SYN, fg.ACK, fg.FIN, fg.RST, fg.PSH
    udp = fg.udp_frame("10.0.0.7", 5000, "1.1.1.7", 443, 40)
    b1 = [a_o(S), b_o(F | A), a_b(S | A), c_o(R), a_o(A), d_o(S | F), e_o(S), f_o(S), f_o(S | A), udp,
          a_o(P | A, 100), a_b(P | A, 50), f_o(F | A), f_b(A), b_o(S), g_o(S), g_o(S | A), g_o(A, 5), g_o(F | A),
          h_o(S), h_o(S | A), h_b(S | A)]
    b2 = [e_b(S | A), a_o(F | A), f_o(A, 10), udp, b_b(S | A), a_b(F | A), g_b(F | A)]
    b3 = [e_b(R), e_o(A), a_o(A), f_b(F | A), h_o(S | R), h_b(A)]
    return [fg.pack(b1), fg.pack(b2), fg.pack([]), fg.pack(b3)]


# conn_state per flow (last octet of the canonical source, protocol); the oracle agrees, and
# each follows determine_conn_state by hand as commented in hand_batches()
HAND_STATES = {(1, 6): "-", (2, 6): "-", (3, 6): "REJ", (4, 6): "S0", (5, 6): "REJ", (6, 6): "S0",
               (8, 6): "S0", (9, 6): "S1", (7, 17): None}


def test_history_hand_sequences():
    for seg in (False, True):
        gf = _run(hand_batches(), seg=seg)
        got = {(int(r["src_ip"][0]) & 0xFF, int(r["protocol"])): N.CONN_STATES[int(r["conn_state"])] for r in gf}
        assert got == HAND_STATES, got


def test_history_parsed_path_record_order(gpu_capture):
    """fb_process_parsed: history follows record (call) order, positions carry the caller's
    pkt_index even when it is not increasing."""
    from flodbadd_amd.sessions import packets_to_parsed, records_to_packets
    frames, offs = synth.generate(4, 40000, first=0, zipf=1, zipf_s=1.1)
    r_out, _, _, _ = coracle.parse_classify(coracle.make_cfg(2), frames, offs)
    parsed = packets_to_parsed(records_to_packets(r_out[:20000]))
    parsed["pkt_index"] = (np.arange(len(parsed), dtype=np.uint32) * 7919) % 100003  # scrambled
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 20, track_history=True)
    flows = coracle.Flows()
    try:
        for half in (parsed[:12000], parsed[12000:]):
            g = cap.process_parsed(half)
            o_out, _, _ = coracle.process_parsed(coracle.make_cfg(2), half)
            assert g.records.tobytes() == o_out.tobytes()
            flows.update(o_out)
        _check_tables(cap, flows)
    finally:
        cap.close()


def test_history_buffer_contract(gpu_capture):
    """fb_flow_history_dev right after a clear (no update) reports 0 characters."""
    gpu_capture.clear_all_sessions()
    d_n = N.DeviceBuffer(4)
    N.check(N.gpu_lib().fb_flow_history_dev(gpu_capture.ctx, None, None, d_n.ptr, None))
    assert int(d_n.download(np.zeros(1, dtype=np.uint32))[0]) == 0


@pytest.mark.parametrize("seg", [False, True], ids=["dense", "seg"])
def test_history_hot_flows_combined(seg):
    """Hot (chunk, partition) groups are combined per key before the apply (k_flow_combine):
    four flows carry most of each batch with random TCP flags in both directions (S, SA, A, PA,
    F, R ... so first S/s/H/h, the first FIN/RST and conn_state all come out of partial
    reductions), interleaved with cold flows, a small table (many keys per partition) and three
    batches so the ordered state also spans updates."""
    import random
    rnd = random.Random(7)
    hot = [("10.0.0.%d" % (i + 1), 40000 + i, "93.184.216.%d" % (i + 1), 443) for i in range(4)]
    flag_set = [fg.SYN, fg.SYN | fg.ACK, fg.ACK, fg.ACK | fg.PSH, fg.FIN | fg.ACK, fg.RST, fg.RST | fg.ACK, 0]
    batches = []
    for b in range(3):
        frames = []
        for k in range(40000):
            if rnd.random() < 0.8:
                s, sp, d, dp = hot[rnd.randrange(4)]
                fl = rnd.choices(flag_set, weights=[1, 1, 60, 30, 1, 0.5, 0.5, 1])[0]
                if rnd.random() < 0.5:
                    s, sp, d, dp = d, dp, s, sp
                frames.append(fg.tcp_frame(s, sp, d, dp, fl, rnd.randrange(64)))
            else:
                c = rnd.randrange(3000)
                frames.append(fg.tcp_frame("172.16.%d.%d" % (c >> 8, c & 255), 1024 + c, "8.8.4.4", 53 + 1 + c % 7,
                                           rnd.choice(flag_set), 10))
        batches.append(fg.pack(frames))
    gf = _run(batches, seg=seg, capacity=1 << 14)
    assert (gf["hist_len"] > 10000).sum() == 4


def test_history_combine_table_overflow():
    """A hot group with more distinct keys than k_flow_combine's LDS table holds (256): 32
    partitions, ~400 cold flows each and one hot flow at 12 % put ~270 keys into the hot
    partition's group per chunk, so some keys stay plain entries beside the combined ones."""
    import random
    rnd = random.Random(11)
    flag_set = [fg.SYN, fg.SYN | fg.ACK, fg.ACK, fg.ACK | fg.PSH, fg.FIN | fg.ACK, fg.RST]
    batches = []
    for b in range(2):
        frames = []
        for k in range(49152):
            fl = rnd.choices(flag_set, weights=[1, 1, 60, 30, 1, 1])[0]
            if rnd.random() < 0.12:
                frames.append(fg.tcp_frame("10.9.8.7", 50000, "93.184.216.34", 443, fl, 20))
            else:
                c = rnd.randrange(13000)
                frames.append(fg.tcp_frame("172.%d.%d.%d" % (16 + (c >> 16), (c >> 8) & 255, c & 255), 2000 + c % 50000,
                                           "9.9.9.9", 443, fl, 5))
        batches.append(fg.pack(frames))
    # precondition (host-side hash): a hot group of the first batch holds > 256 distinct keys
    lib = N.gpu_lib()
    recs = coracle.parse_classify(coracle.make_cfg(2), *batches[0])[0]
    groups = {}
    for i in range(len(recs)):
        h = lib.fb_flow_hash(N.ptr(recs[i: i + 1]))
        groups.setdefault((i // 20480, h >> 59), []).append(recs[i: i + 1].tobytes()[:40])
    assert max(len(set(v)) for v in groups.values() if len(v) >= 2048) > 256
    gf = _run(batches, capacity=1 << 14)
    assert (gf["hist_len"] > 10000).sum() == 1


def test_history_split_list_overflow():
    """More partitions over kHistSplitEntries (8192 entries to read) than the split list holds
    (kHistListCap = 256): a 2^18-slot table has 512 partitions and a 5M-record batch over 100K
    flows puts ~9,800 records into each, so 256 partitions are split by chunk blocks and the rest
    go whole to k_hist_general's slow list; every flow's history string equals the oracle's."""
    big = synth.generate(2, 5_000_000, first=0, n_flows=100_000)
    tail = synth.generate(2, 300_000, first=5_000_000, n_flows=100_000)
    # precondition (host-side hash): > 256 of the 512 partitions hold > 8192 records
    lib = N.gpu_lib()
    recs = coracle.parse_classify(coracle.make_cfg(2), *big)[0]
    keys = np.ascontiguousarray(np.ascontiguousarray(recs).view(np.uint8).reshape(len(recs), -1)[:, :40])
    uniq, first, counts = np.unique(keys.view("V40").ravel(), return_index=True, return_counts=True)
    per_part = np.zeros(512, dtype=np.int64)
    for i, c in zip(first, counts):
        per_part[lib.fb_flow_hash(N.ptr(recs[i: i + 1])) >> 55] += c
    assert (per_part > 8192).sum() > 256, per_part
    del recs, keys, uniq
    gf = _run([big, tail], seg=True, capacity=1 << 18)
    assert len(gf) > 90_000 and (gf["hist_len"] > 20).any()


def test_k2_heavy_partition_list_overflow():
    """More heavy partitions than K2's leading list holds (kK2Lead = 256, fb_flow.hip K1t / K2): a
    2^19-slot table has 1,024 partitions; 400 warm flows carry 10K records each of a 5M-record batch
    (~41 per bucketing chunk, under k_flow_combine's minimum, so they stay plain entries) and 100K
    cold flows the rest, so ~330 partitions pass twice the mean -- the first 256 go to K2's leading
    workgroups, the others stay with the later ones.  A second, cold-only batch then has no heavy
    partition (the list and its flags must be cleared per update).  Every flow row and history
    equals the oracle's."""
    rnd = np.random.default_rng(5)
    n_warm, per_warm, n_cold, n = 400, 10_000, 100_000, 5_000_000
    tmpl = []  # two 60-byte frames per flow: ACK, PSH | ACK
    for i in range(n_warm + n_cold):
        src = ("10.%d.%d.%d" if i < n_warm else "172.%d.%d.%d") % (16 + (i >> 16), (i >> 8) & 255, i & 255)
        for fl in (fg.ACK, fg.ACK | fg.PSH):
            tmpl.append(fg.tcp_frame(src, 1024 + i % 60000, "93.184.216.34", 443, fl, 6))
    L = len(tmpl[0])
    assert all(len(t) == L for t in tmpl)
    T = np.frombuffer(b"".join(tmpl), dtype=np.uint8).reshape(-1, L)
    del tmpl

    def batch(ids):
        sel = ids * 2 + rnd.integers(0, 2, len(ids))
        return np.ascontiguousarray(T[sel]).reshape(-1), (np.arange(len(ids) + 1, dtype=np.uint64) * L).astype(np.uint32)

    ids = np.concatenate([np.repeat(np.arange(n_warm), per_warm),
                          rnd.integers(n_warm, n_warm + n_cold, n - n_warm * per_warm)])
    rnd.shuffle(ids)
    big = batch(ids)
    cold = batch(rnd.integers(n_warm, n_warm + n_cold, 1_000_000))
    # precondition (host-side hash): more partitions than the list holds pass K1t's threshold
    lib = N.gpu_lib()
    cfg = coracle.make_cfg(2)
    keys = coracle.parse_classify(cfg, T[0::2].reshape(-1), (np.arange(len(T) // 2 + 1, dtype=np.uint64) * L).astype(np.uint32))[0]
    part = np.array([lib.fb_flow_hash(N.ptr(keys[i: i + 1])) >> 54 for i in range(len(keys))])
    per_part = np.bincount(part, weights=np.bincount(ids, minlength=len(keys)), minlength=1024)
    lead_min = 2 * ((n + 20479) // 20480) * 20480 // 1024
    assert (per_part >= lead_min).sum() > 256, (per_part >= lead_min).sum()
    del keys, ids
    gf = _run([big, cold], seg=True, capacity=1 << 19)
    assert len(gf) == n_warm + n_cold


def test_history_full_size_zipf():
    """The bench's skewed C4 batch at full size (10,485,760 IMIX frames, Zipf(1.1)) and a 1M
    follow-up: every flow's history string, conn_state and ordered fields equal the oracle's --
    the hottest flows' partitions split by chunk blocks, thousands of combined groups read back in
    record order through e_sort."""
    batches = [synth.generate(4, 10 * (1 << 20), first=0, zipf=1, zipf_s=1.1),
               synth.generate(4, 1 << 20, first=10 * (1 << 20), zipf=1, zipf_s=1.1)]
    gf = _run(batches, seg=True, capacity=1 << 22)
    assert (gf["hist_len"] > 100000).any()
