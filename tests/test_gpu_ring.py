"""Host ingest ring (fb_ring_*) against the oracle: frames pushed one by one,
in blocks and through zero-copy reservations come out as the same per-batch results as the
oracle run over the same batch cuts -- cumulative stats, the session table (counters and ordered
state) and the DNS side records with their payload bytes -- with fewer pinned slots than batches
(the producer waits for the oldest batch instead of dropping)."""
import ctypes as C

import numpy as np
import pytest

import framegen as fg
from flodbadd_amd import _native as N
from flodbadd_amd import synth
from oracle import coracle
from test_gpu_parity import rows_sorted

pytestmark = pytest.mark.gpu


def _ring(cap, slots, max_packets, max_bytes, flags=0, copy_threads=0):
    cfg = N.FbRingConfig(slots, max_packets, max_bytes, flags, copy_threads)
    r = N.gpu_lib().fb_ring_create(cap.ctx, C.byref(cfg))
    assert r, N.gpu_lib().fb_last_error()
    return C.c_void_p(r)


def _poll_dns(lib, r):
    out = np.zeros(1 << 16, dtype=N.RING_DNS_DTYPE)
    buf = np.zeros(1 << 22, dtype=np.uint8)
    n, nb = C.c_uint32(), C.c_uint64()
    N.check(lib.fb_ring_poll_dns(r, N.ptr(out), len(out), N.ptr(buf), buf.nbytes, C.byref(n), C.byref(nb)))
    recs = out[: n.value]
    return [(int(d["packet_seq"]), int(d["protocol"]), bytes(buf[d["payload_offset"]: d["payload_offset"] + d["payload_length"]]))
            for d in recs]


def _oracle_batches(frames, offs, per_batch, flows):
    """The oracle over the ring's batch cuts (every `per_batch` frames); returns totals + DNS."""
    cfg = coracle.make_cfg(2)
    n = len(offs) - 1
    tot = np.zeros(1, dtype=N.STATS_DTYPE)
    dns = []
    for a in range(0, n, per_batch):
        b = min(n, a + per_batch)
        o = offs[a: b + 1] - offs[a]
        fr = frames[offs[a]: offs[b]]
        out, d, _, st = coracle.parse_classify(cfg, fr, o)
        flows.update(out, st)
        for k in N.STATS_FIELDS:
            if not k.startswith("reserved"):
                tot[0][k] += st[0][k]
        for x in d:
            pl = bytes(fr[x["payload_offset"]: x["payload_offset"] + x["payload_length"]])
            dns.append((a + int(x["pkt_index"]), int(x["protocol"]), pl))
    return tot, dns


@pytest.mark.parametrize("how", ["block", "push", "reserve", "block_mt"])
def test_ring_vs_oracle(gpu_capture, how):
    """block_mt: 150k frames in blocks split over 5 copy threads (fb_ring_config.copy_threads; runs of
    more than 1 MB are copied by frame ranges, a block of 65,536+ frames is validated by ranges)."""
    frames, offs = synth.generate(3, 150000 if how == "block_mt" else 20000, first=11)
    extra, eo = fg.pack([f for _, f in fg.edge_cases()])
    frames = np.concatenate([frames, extra])
    offs = np.concatenate([offs, offs[-1] + eo[1:]]).astype(np.uint32)
    n = len(offs) - 1
    per = 3000 if how != "block_mt" else 40000  # 7 (4) batches through 3 pinned slots
    lib = N.gpu_lib()
    gpu_capture.clear_all_sessions()
    r = _ring(gpu_capture, 3, per, 64 << 20, copy_threads=5 if how == "block_mt" else 0)
    try:
        if how in ("block", "block_mt"):
            cut = 5000 if how == "block" else 70001
            N.check(lib.fb_ring_push_block(r, N.ptr(frames), N.ptr(offs), cut))
            rest = np.ascontiguousarray(offs[cut:] - offs[cut], dtype=np.uint32)  # kept alive for the call
            tail = frames[offs[cut]:]
            N.check(lib.fb_ring_push_block(r, N.ptr(tail), N.ptr(rest), n - cut))
        elif how == "push":
            for i in range(n):
                f = np.ascontiguousarray(frames[offs[i]: offs[i + 1]])
                N.check(lib.fb_ring_push(r, N.ptr(f), len(f)))
        else:
            for i in range(n):
                ln = int(offs[i + 1] - offs[i])
                p = lib.fb_ring_reserve(r, ln)
                assert p
                C.memmove(p, frames[offs[i]: offs[i + 1]].ctypes.data, ln)
        N.check(lib.fb_ring_sync(r))
        tot = np.zeros(1, dtype=N.STATS_DTYPE)
        nb, nf = C.c_uint64(), C.c_uint64()
        N.check(lib.fb_ring_stats(r, N.ptr(tot), C.byref(nb), C.byref(nf)))
        got_dns = _poll_dns(lib, r)
    finally:
        lib.fb_ring_destroy(r)
    flows = coracle.Flows()
    r_tot, r_dns = _oracle_batches(frames, offs, per, flows)
    assert nf.value == n and nb.value == (n + per - 1) // per
    for k in N.STATS_FIELDS:
        if not k.startswith("reserved"):
            assert int(tot[0][k]) == int(r_tot[0][k]), k
    assert got_dns == r_dns
    assert rows_sorted(gpu_capture.export_flows()) == rows_sorted(flows.export_sorted())
    gpu_capture.clear_all_sessions()


def test_ring_bad_arguments(gpu_capture):
    lib = N.gpu_lib()
    bad = N.FbRingConfig(1, 100, 1 << 20, 0, 0)
    assert not lib.fb_ring_create(gpu_capture.ctx, C.byref(bad))
    r = _ring(gpu_capture, 2, 4, 256)
    try:
        big = np.zeros(300, dtype=np.uint8)
        assert lib.fb_ring_push(r, N.ptr(big), 300) == N.FB_ERR_INVAL  # frame > max_bytes
        offs = np.array([0, 10, 5], dtype=np.uint32)
        assert lib.fb_ring_push_block(r, N.ptr(big), N.ptr(offs), 2) == N.FB_ERR_INVAL
        N.check(lib.fb_ring_sync(r))  # nothing pushed: no batch
        nb = C.c_uint64()
        N.check(lib.fb_ring_stats(r, None, C.byref(nb), None))
        assert nb.value == 0
    finally:
        lib.fb_ring_destroy(r)
    # the range-split validation of a multi-threaded ring: a decrease deep in a large block is
    # found and nothing of the block is taken
    r = _ring(gpu_capture, 2, 1 << 17, 1 << 24, copy_threads=4)
    try:
        n = 100000
        offs = np.arange(n + 1, dtype=np.uint32) * 64
        offs[77777] = offs[77776] - 1
        fr = np.zeros(n * 64, dtype=np.uint8)
        assert lib.fb_ring_push_block(r, N.ptr(fr), N.ptr(offs), n) == N.FB_ERR_INVAL
        assert b"77776" in lib.fb_last_error()
        N.check(lib.fb_ring_sync(r))
        nb, nf = C.c_uint64(), C.c_uint64()
        N.check(lib.fb_ring_stats(r, None, C.byref(nb), C.byref(nf)))
        assert nb.value == 0 and nf.value == 0
    finally:
        lib.fb_ring_destroy(r)


def test_ingest_ring_wrapper(gpu_capture):
    """flodbadd_amd.capture.IngestRing: per-frame pushes incl. DNS over UDP and TCP, then the
    DNS payloads and totals the oracle gives for the same single batch."""
    from flodbadd_amd.capture import IngestRing
    frames = [fg.udp_frame("10.0.0.2", 5000 + i, "8.8.8.8", 53, 20 + i) for i in range(40)] + \
             [fg.tcp_frame("10.0.0.3", 7000 + i, "1.1.1.1", 443, fg.ACK, 10) for i in range(60)] + \
             [f for _, f in fg.edge_cases()]
    buf, offs = fg.pack(frames)
    gpu_capture.clear_all_sessions()
    ring = IngestRing(gpu_capture, slots=2, max_packets=4096, max_bytes=1 << 20)
    try:
        for f in frames:
            ring.push(f)
        ring.sync()
        st, nb, nf = ring.stats()
        dns = ring.poll_dns()
    finally:
        ring.close()
    flows = coracle.Flows()
    r_tot, r_dns = _oracle_batches(buf, offs, 4096, flows)
    assert nb == 1 and nf == len(frames)
    assert st["n_dns"] == int(r_tot[0]["n_dns"]) and st["n_session"] == int(r_tot[0]["n_session"])
    assert [(s, p, pl) for s, p, _, pl in dns] == r_dns
    gpu_capture.clear_all_sessions()
