#!/usr/bin/env python3
"""bench.py -- Mpackets/s of device-resident parse + 5-tuple classify on MI355X.

One step = one pass of the hot path (k_parse_seg: parse_packet_pcap + the per-packet part of
process_parsed_packet, src/packets.rs:202-802) over one batch of synthetic frames that is already
resident in HBM.  Default workload = BASELINE.json configs[1] (C2): 1,048,576 x 64-B IPv4/TCP
frames per GPU.  Batches rotate over R distinct device buffer sets (C2: 32, 4 GB) so the working
set exceeds the 256 MB Infinity Cache and the timing is HBM-bound, not MALL-bound; consecutive
steps share launches of up to 32 batches (fb_parse_classify_seg_batches_dev), split evenly.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) every process is one rank;
`python3 bench.py --gpus N` with no WORLD_SIZE spawns the N rank processes itself (spawn_ranks,
before anything touches the GPU) and exits with their status.  Packets are sharded by index (each
rank owns the contiguous range [rank*n, (rank+1)*n) of the virtual batch) with no data-path
collective ("scaling": "weak"); torch.distributed (gloo, CPU) only provides the barrier and the
max over ranks of the timed region; the C5 extra exchanges the per-flow table over RCCL.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MAX_SEG_BATCHES = 32  # FB_MAX_SEG_BATCHES, include/flodbadd_gpu.h
WORKLOADS = {
    2: "C2: 1,048,576 x 64-B IPv4/TCP frames per GPU, device-resident (BASELINE configs[1])",
    3: "C3: 1,048,576-frame IMIX 64/576/1500 (7:4:1), IPv4+IPv6, TCP+UDP per GPU, device-resident",
    4: "C4: 10,485,760-frame IMIX batch per GPU, device-resident, + session-table upsert with per-flow counters (pool 2^20)",
}


def algorithmic_bytes(offsets, n_session, n_dns):
    """B = sum(min(caplen,128)) + 4 B offset per frame (+1 sentinel)
    + 56 B per emitted session record + 16 B per DNS record (no class array requested)."""
    caplen = np.diff(offsets.astype(np.int64))
    return int(np.minimum(caplen, 128).sum()) + 4 * len(offsets) + 56 * int(n_session) + 16 * int(n_dns)


def plan_launches(k, bpl):
    """Split k consecutive steps into ceil(k / bpl) launches of near-equal size (a short final
    launch would pay the per-launch start-up and tail for a fraction of the batches)."""
    if k <= 0:
        return []
    m = -(-k // bpl)
    q, r = divmod(k, m)
    return [q + 1] * r + [q] * (m - r)


def run_config(N, lib, ctx, config_id, n, steps, warmup, rotate, rank, world, dist, flow=False, mode="seg", bpl=1,
               synth_kw=None, pipelined=False, stage_extras=True, records=True, timed=False):
    """Time `steps` steps (one step = one batch through the hot path).  mode "seg":
    fb_parse_classify_seg_dev (records compacted per 64-frame wavefront segment, no
    cross-workgroup dependency); mode "dense": fb_parse_classify_dev (the same kernel + the
    batch-wide compaction of fb_compact.hip).  flow=True (C4): fb_process[_seg]_dev -- parse +
    classify, then the session-table upsert -- with the context's stage event recorded between
    the two, so each stage is timed inside the fused call.
    bpl > 1 (mode "seg", no flow): consecutive steps share launches of up to bpl batches
    (fb_parse_classify_seg_batches_dev; each batch its own outputs and stats), split evenly by
    plan_launches.  Batch i uses buffer set i % rotate, so rotate >= bpl keeps the batches of a
    launch distinct.  pipelined (flow, mode "seg"): fb_process_seg_async_dev -- each batch's table
    update on the context's own stream while the next batch is parsed (rotate >= 2 buffer sets),
    joined (fb_flow_join) inside the timed region.  records=False (flow, mode "seg"): the fused calls
    keep only the session table (fb_set_session_records 0), as the reference's capture loop does."""
    from flodbadd_amd import synth
    frames, offs = synth.generate(config_id, n, first=rank * n, **(synth_kw or {}))
    nbytes = frames.nbytes
    stream = N.Stream()
    nseg = (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
    bufs = []
    for _ in range(rotate):
        d_fr = N.DeviceBuffer(nbytes).upload(frames)
        d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
        if mode == "seg":
            d_out = N.DeviceBuffer(nseg * N.SEG_BYTES)
            d_dns = N.DeviceBuffer(nseg * 4)  # the segment counts
        else:
            d_out = N.DeviceBuffer(n * N.PKT_OUT_DTYPE.itemsize)
            d_dns = N.DeviceBuffer(n * N.DNS_OUT_DTYPE.itemsize)
        d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        bufs.append((d_fr, d_off, d_out, d_dns, d_st))
    # timed contexts (flow): every buffer set's frame capture times (~2 us apart, set j one second later)
    d_ts = [N.DeviceBuffer(8 * n).upload(
        (1_700_000_000 * 10 ** 9 + j * 10 ** 9 + 2000 * np.arange(n, dtype=np.uint64)).astype(np.uint64))
        for j in range(rotate)] if timed else None

    def descriptors(first, count):
        d = np.zeros(count, dtype=N.SEG_BATCH_DTYPE)
        for t in range(count):
            d_fr, d_off, d_out, d_seg, d_st = bufs[(first + t) % rotate]
            d[t] = (d_fr.ptr.value, nbytes, d_off.ptr.value, n, 0, d_out.ptr.value, d_seg.ptr.value, 0, d_st.ptr.value)
        return d

    keep = []  # descriptor arrays referenced by address

    def plan(k):
        """Launch descriptors of k steps, built before the timed region."""
        if bpl == 1:
            return None
        assert mode == "seg" and not flow and rotate >= bpl, (mode, flow, rotate, bpl)
        out, first = [], 0
        for c in plan_launches(k, bpl):
            d = descriptors(first, c)
            keep.append(d)
            out.append((d.ctypes.data, c))
            first += c
        return out

    def run_steps(k, launches):
        """k steps; returns the number of kernel launches."""
        if launches is None:
            for i in range(k):
                step(i)
            return k
        for d, c in launches:
            rc = lib.fb_parse_classify_seg_batches_dev(ctx, d, c, stream.ptr)
            if rc != 0:
                raise RuntimeError(lib.fb_last_error().decode())
        return len(launches)

    def step(i):
        d_fr, d_off, d_out, d_dns, d_st = bufs[i % rotate]
        if d_ts is not None:
            N.check(lib.fb_set_frame_times(ctx, d_ts[i % rotate].ptr))
        if mode == "seg" and flow:
            # fb_process_seg_dev: parse + session upsert in one call (the parse also hands each
            # record's table partition to the update's histogram pass); pipelined: the async form
            fn = lib.fb_process_seg_async_dev if pipelined else lib.fb_process_seg_dev
            rc = fn(ctx, d_fr.ptr, nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr, None, d_st.ptr, stream.ptr)
        elif mode == "seg":
            rc = lib.fb_parse_classify_seg_dev(ctx, d_fr.ptr, nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr, None,
                                               d_st.ptr, stream.ptr)
        elif flow:
            rc = lib.fb_process_dev(ctx, d_fr.ptr, nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr, None, d_st.ptr,
                                    stream.ptr)
        else:
            rc = lib.fb_parse_classify_dev(ctx, d_fr.ptr, nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr, None,
                                           d_st.ptr, stream.ptr)
        if rc != 0:
            raise RuntimeError(lib.fb_last_error().decode())

    if flow:
        N.check(lib.fb_flow_clear(ctx, stream.ptr))
    N.check(lib.fb_set_session_records(ctx, 1 if records else 0))
    run_steps(warmup, plan(warmup))
    if pipelined:
        N.check(lib.fb_flow_join(ctx, stream.ptr))
    stream.sync()
    st = bufs[0][4].download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)
    if int(st[0]["error"]) or int(st[0]["n_session"]) + int(st[0]["n_dns"]) + int(st[0]["n_drop"]) != n:
        raise RuntimeError("bad batch stats: %s" % st)
    # FB_BENCH_ABLATION: timing-only library variants (tools/build_variants.sh) skip the table check
    if flow and int(st[0]["new_sessions"]) + int(st[0]["updated_sessions"]) != int(st[0]["n_session"]) \
            and not os.environ.get("FB_BENCH_ABLATION"):
        raise RuntimeError("flow upsert lost records: %s" % st)
    ev0, ev1 = N.Event(), N.Event()
    launches = plan(steps)
    if flow and pipelined:
        def run_timed():
            for i in range(steps):
                step(i)
            N.check(lib.fb_flow_join(ctx, stream.ptr))  # the last update is part of the region
            return steps
    elif flow:
        # per step: start, the stage event (recorded by the library between parse and update), end
        evs = [(N.Event(), N.Event(), N.Event()) for _ in range(steps)]

        def run_timed():
            for i in range(steps):
                evs[i][0].record(stream)
                N.check(lib.fb_set_stage_event(ctx, evs[i][1].ptr))
                step(i)
                evs[i][2].record(stream)
            N.check(lib.fb_set_stage_event(ctx, None))
            return steps
    else:
        def run_timed():
            return run_steps(steps, launches)
    if dist:
        dist.barrier()
    stream.sync()
    t0 = time.perf_counter()
    ev0.record(stream)
    n_launch = run_timed()
    ev1.record(stream)
    ev1.wait_spin()  # poll the completion (a blocking wait adds its wake-up latency to the region)
    t1 = time.perf_counter()
    stream.sync()
    if dist:
        dist.barrier()
    elapsed = local_elapsed = t1 - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ev_ms = ev0.elapsed_ms(ev1)
    algo = algorithmic_bytes(offs, st[0]["n_session"], st[0]["n_dns"])
    # make sure the last step's results are sane too
    st2 = bufs[(steps - 1) % rotate][4].download(np.zeros(1, dtype=N.STATS_DTYPE), stream=stream.ptr)
    stage = None
    if flow:
        # after warmup every session exists: the timed steps are all updates
        same = [k for k in st.dtype.names if k not in ("new_sessions", "updated_sessions")]
        assert all(int(st2[0][k]) == int(st[0][k]) for k in same), (st, st2)
        assert int(st2[0]["updated_sessions"]) + int(st2[0]["new_sessions"]) == int(st2[0]["n_session"]) \
        or os.environ.get("FB_BENCH_ABLATION")
        # the parse stage as it runs inside the fused call (for fb_process_seg_dev: the
        # partition-writing instance of k_parse_seg), the update the rest of the step (the
        # pipelined form overlaps them: no split)
        if pipelined:
            stage = dict(parse_ms=None, flow_ms=None)
        else:
            parse_ms = sum(a.elapsed_ms(b) for a, b, _ in evs) / steps
            flow_ms = sum(b.elapsed_ms(c) for _, b, c in evs) / steps
            stage = dict(parse_ms=parse_ms, flow_ms=flow_ms)
    if flow and stage_extras:
        # ordered per-flow history of the last update (fb_flow_history_dev: keys + stable radix sort)
        slots = n if mode == "dense" else (n + 63) // 64 * 64
        d_h, d_s, d_n = N.DeviceBuffer(slots), N.DeviceBuffer(4 * slots), N.DeviceBuffer(4)
        h0, h1 = N.Event(), N.Event()
        N.check(lib.fb_flow_history_dev(ctx, d_h.ptr, d_s.ptr, d_n.ptr, stream.ptr))  # scratch allocation
        h0.record(stream)
        for _ in range(5):
            N.check(lib.fb_flow_history_dev(ctx, d_h.ptr, d_s.ptr, d_n.ptr, stream.ptr))
        h1.record(stream)
        stage["history_ms"] = h0.elapsed_ms(h1) / 5
        stage["history_chars"] = int(d_n.download(np.zeros(1, dtype=np.uint32), stream=stream.ptr)[0])
        for x in (d_h, d_s, d_n):
            x.free()
        cnt = C.c_uint64()
        N.check(lib.fb_flow_count(ctx, C.byref(cnt), stream.ptr))
        stage["flows"] = int(cnt.value)
        stage.update(enrich_timing(N, lib, ctx, int(cnt.value), stream))
        stage.update(dns_timing(N, lib, ctx, stream))
    if not flow:
        assert st2.tobytes() == st.tobytes()
    N.check(lib.fb_set_session_records(ctx, 1))
    if not records:  # no session record is written: the parse's bytes are the headers, offsets, DNS records
        algo -= 56 * int(st[0]["n_session"])
    for b in bufs + (d_ts or []):
        for x in (b if isinstance(b, tuple) else (b,)):
            x.free()
    return dict(frames=frames, offs=offs, elapsed=elapsed, local_elapsed=local_elapsed, ev_ms=ev_ms,
                algo_bytes=algo, stage=stage,
                host_us=round((t1 - t0) * 1e6 - ev_ms * 1e3, 1),
                launches=n_launch, stats={k: int(st[0][k]) for k in ("n_session", "n_dns", "n_drop", "n_filtered")})


def queue_line(N, lib, ctx, config_id, n, steps, warmup, rotate, depth=8):
    """One batch per call without a launch per batch: the resident queue-fed parse (fb_seg_queue_*,
    k_parse_seg_queue).  The same device-resident workload as the main line (rotate distinct batch
    buffer sets); the host submits one batch per call and the timed region runs from the first
    submission to the observed completion of the last (host wall clock: the queue's kernel runs on
    its own stream).  Every batch's stats are checked against a plain fb_parse_classify_seg_dev."""
    from flodbadd_amd import synth
    frames, offs = synth.generate(config_id, n, first=0)
    nseg = (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
    sets, descs = [], []
    for _ in range(rotate):
        b = (N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
             N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize))
        d = np.zeros(1, dtype=N.SEG_BATCH_DTYPE)
        d[0] = (b[0].ptr.value, frames.nbytes, b[1].ptr.value, n, 0, b[2].ptr.value, b[3].ptr.value, 0, b[4].ptr.value)
        sets.append(b)
        descs.append(d)
    # the expected stats: one plain launch into the first set
    ref = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
    b = sets[0]
    N.check(lib.fb_parse_classify_seg_dev(ctx, b[0].ptr, frames.nbytes, b[1].ptr, n, b[2].ptr, b[3].ptr, None, ref.ptr, None))
    expect = ref.download(np.zeros(1, dtype=N.STATS_DTYPE))
    N.check(lib.fb_stream_sync(None))
    q = lib.fb_seg_queue_create(ctx, depth, 0)
    if not q:
        raise RuntimeError("fb_seg_queue_create: %s" % lib.fb_last_error().decode())
    q = C.c_void_p(q)
    ptrs = [C.c_void_p(d.ctypes.data) for d in descs]
    t = C.c_uint64()
    submit, wait = lib.fb_seg_queue_submit, lib.fb_seg_queue_wait
    try:
        for i in range(warmup):
            N.check(submit(q, ptrs[i % rotate], C.byref(t)))
        N.check(wait(q, t.value))
        t0 = time.perf_counter()
        for i in range(steps):
            rc = submit(q, ptrs[i % rotate], C.byref(t))
            if rc:
                N.check(rc)
        N.check(wait(q, t.value))
        t1 = time.perf_counter()
    finally:
        N.check(lib.fb_seg_queue_destroy(q))
    for k in range(min(rotate, steps)):
        got = sets[k][4].download(np.zeros(1, dtype=N.STATS_DTYPE))
        if got.tobytes() != expect.tobytes():
            raise RuntimeError("queue batch %d stats differ: %s vs %s" % (k, got, expect))
    for b in sets:
        for x in b:
            x.free()
    el = t1 - t0
    return dict(value=round(n * steps / el / 1e6, 2), unit="Mpackets/s", ms_per_step=round(el * 1e3 / steps, 4),
                steps=steps, depth=depth,
                note="fb_seg_queue_submit per batch into the resident k_parse_seg_queue kernel; host wall clock "
                     "from the first submission to the last batch's completion word (a batch takes ~85 us from "
                     "submission to completion, DESIGN 3.7: the first batches' fill is inside the timed region)")


def queue_table_line(N, lib, ctx, n=1 << 20, steps=100, warmup=8, rotate=4, depth=4):
    """One batch per call WITH the session-table upsert through the resident queue: a queue created
    shared (FB_QUEUE_SHARED: one workgroup on each of an eighth of the CUs) parses C4-mix batches of n frames while each
    completed batch is applied to the context's table on a stream of its own (fb_flow_update_seg_dev
    beside the resident kernel); `rotate` device buffer sets, a set resubmitted only after its last
    update completed.  Host wall clock from the first submission to the last update's completion."""
    from flodbadd_amd import synth
    frames, offs = synth.generate(4, n, first=0)
    nseg = (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
    sets, descs = [], []
    for _ in range(rotate):
        b = (N.DeviceBuffer(frames.nbytes).upload(frames), N.DeviceBuffer(offs.nbytes).upload(offs),
             N.DeviceBuffer(nseg * N.SEG_BYTES), N.DeviceBuffer(nseg * 4), N.DeviceBuffer(N.STATS_DTYPE.itemsize))
        d = np.zeros(1, dtype=N.SEG_BATCH_DTYPE)
        d[0] = (b[0].ptr.value, frames.nbytes, b[1].ptr.value, n, 0, b[2].ptr.value, b[3].ptr.value, 0, b[4].ptr.value)
        sets.append(b)
        descs.append(d)
    upd = N.Stream()
    evs = [N.Event() for _ in range(rotate)]
    N.check(lib.fb_flow_clear(ctx, None))
    N.check(lib.fb_stream_sync(None))
    q = lib.fb_seg_queue_create_ex(ctx, depth, 0, N.FB_QUEUE_SHARED)
    if not q:
        raise RuntimeError("fb_seg_queue_create_ex: %s" % lib.fb_last_error().decode())
    q = C.c_void_p(q)
    ptrs = [C.c_void_p(d.ctypes.data) for d in descs]
    tk = C.c_uint64()
    submit, wait = lib.fb_seg_queue_submit, lib.fb_seg_queue_wait

    def run(k0, count):
        """Batches k0 .. k0 + count - 1: submit batch i, then apply batch i - 1 once it completed."""
        tickets = {}
        for i in range(k0, k0 + count + 1):
            if i < k0 + count:
                if i - k0 >= rotate:
                    evs[i % rotate].wait_spin()  # the set's previous batch is applied
                N.check(submit(q, ptrs[i % rotate], C.byref(tk)))
                tickets[i] = tk.value
            if i > k0:
                j = i - 1
                N.check(wait(q, tickets.pop(j)))
                b = sets[j % rotate]
                N.check(lib.fb_flow_update_seg_dev(ctx, b[2].ptr, b[3].ptr, n, b[4].ptr, upd.ptr))
                evs[j % rotate].record(upd)
        upd.sync()
    try:
        run(0, warmup)
        t0 = time.perf_counter()
        run(warmup, steps)
        el = time.perf_counter() - t0
    finally:
        N.check(lib.fb_seg_queue_destroy(q))
    st = sets[(warmup + steps - 1) % rotate][4].download(np.zeros(1, dtype=N.STATS_DTYPE))
    cnt = C.c_uint64()
    N.check(lib.fb_flow_count(ctx, C.byref(cnt), None))
    for b in sets:
        for x in b:
            x.free()
    if int(st[0]["error"]) or int(st[0]["new_sessions"]) + int(st[0]["updated_sessions"]) != int(st[0]["n_session"]):
        raise RuntimeError("queue + table batch stats inconsistent: %s" % st)
    N.check(lib.fb_flow_clear(ctx, None))
    return dict(value=round(n * steps / el / 1e6, 2), unit="Mpackets/s", ms_per_batch=round(el * 1e3 / steps, 4),
                steps=steps, frames_per_batch=n, flows_in_table=int(cnt.value),
                note="C4-mix batches one per call through a shared resident queue (FB_QUEUE_SHARED), each "
                     "completed batch applied to the session table on its own stream beside it")


def enrich_timing(N, lib, ctx, flows, stream, reps=5):
    """New-session enrichment (fb_flow_enrich_dev) over every flow of the C4 table against
    IPtoASN-sized synthetic tables: 500k IPv4 + 100k IPv6 ASN ranges, 50k blacklist ranges in 32
    lists (deterministic)."""
    rng = np.random.default_rng(0xA5A5)

    def ranges(n, v6):
        t = np.zeros(n, dtype=N.ASN_RANGE_DTYPE)
        if v6:
            hi = np.sort(rng.integers(0x20000000, 0x2FFFFFFF, n, dtype=np.uint64)).astype(np.uint32)
            t["start"][:, 0] = hi
            t["end"][:, 0] = hi
            t["end"][:, 1:] = 0xFFFFFFFF
        else:
            st = np.sort(rng.choice(np.uint64(1 << 32) - np.uint64(1 << 16), n, replace=False)).astype(np.uint64)
            t["start"][:, 0] = st.astype(np.uint32)
            t["end"][:, 0] = (st + rng.integers(0, 4096, n).astype(np.uint64)).astype(np.uint32)
        t["as_number"] = rng.integers(1, 400000, n)
        t["record"] = np.arange(n)
        return t
    a4, a6 = ranges(500000, False), ranges(100000, True)
    bl = np.zeros(50000, dtype=N.CIDR_DTYPE)
    bl["family"] = 2
    bl["addr"][:, 0] = rng.integers(0, 1 << 32, len(bl), dtype=np.uint64).astype(np.uint32)
    bl["prefix"] = rng.choice([16, 20, 24, 28, 32], len(bl))
    bl["list"] = rng.integers(0, 32, len(bl))
    N.check(lib.fb_set_asn_tables(ctx, N.ptr(a4), len(a4), N.ptr(a6), len(a6)))
    N.check(lib.fb_set_blacklists(ctx, N.ptr(bl), len(bl)))
    d_out, d_n = N.DeviceBuffer(max(flows, 1) * N.FLOW_ENRICH_DTYPE.itemsize), N.DeviceBuffer(8)
    e0, e1 = N.Event(), N.Event()
    N.check(lib.fb_flow_enrich_dev(ctx, 0, d_out.ptr, flows, d_n.ptr, stream.ptr))
    e0.record(stream)
    for _ in range(reps):
        N.check(lib.fb_flow_enrich_dev(ctx, 0, d_out.ptr, flows, d_n.ptr, stream.ptr))
    e1.record(stream)
    ms = e0.elapsed_ms(e1) / reps
    got = int(d_n.download(np.zeros(1, dtype=np.uint64), stream=stream.ptr)[0])
    N.check(lib.fb_set_asn_tables(ctx, None, 0, None, 0))
    N.check(lib.fb_set_blacklists(ctx, None, 0))
    for b in (d_out, d_n):
        b.free()
    return dict(enrich_ms=round(ms, 4), enrich_flows=got, enrich_Mflows_s=round(got / ms / 1e3, 1),
                enrich_tables="500k v4 + 100k v6 ASN ranges, 50k blacklist ranges / 32 lists")


def dns_timing(N, lib, ctx, stream, n=1 << 20, reps=10):
    """DNS divert parse (fb_dns_parse_dev) over a device-resident batch of 1M
    port-53 payloads (synth.dns_workload: queries, reverse lookups, CNAME + A/AAAA responses)."""
    from flodbadd_amd import synth
    payload, rec = synth.dns_workload(n)
    d_fr = N.DeviceBuffer(payload.nbytes).upload(payload)
    d_dns = N.DeviceBuffer(rec.nbytes).upload(rec)
    d_msg = N.DeviceBuffer(n * N.DNS_MSG_DTYPE.itemsize)
    d_names = N.DeviceBuffer(n * N.FB_DNS_MAX_NAME)
    d_addrs = N.DeviceBuffer(n * N.FB_DNS_MAX_ADDRS * N.FB_IP_DTYPE.itemsize)

    def call():
        N.check(lib.fb_dns_parse_dev(ctx, d_fr.ptr, payload.nbytes, d_dns.ptr, n, None, d_msg.ptr, d_names.ptr,
                                     d_addrs.ptr, stream.ptr))
    call()
    e0, e1 = N.Event(), N.Event()
    e0.record(stream)
    for _ in range(reps):
        call()
    e1.record(stream)
    ms = e0.elapsed_ms(e1) / reps
    msgs = d_msg.download(np.zeros(n, dtype=N.DNS_MSG_DTYPE), stream=stream.ptr)
    ok = int((msgs["status"] == 0).sum())
    for b in (d_fr, d_dns, d_msg, d_names, d_addrs):
        b.free()
    return dict(dns_parse_ms=round(ms, 4), dns_msgs=n, dns_ok=ok, dns_Mmsgs_s=round(n / ms / 1e3, 1),
                dns_payload_GBs=round(payload.nbytes / ms / 1e6, 1))


def host_inclusive(N, lib, ctx, frames, offs, calls=20):
    """fb_parse_classify from PINNED host buffers to pinned host outputs: H2D of frames+offsets,
    the kernel, D2H of records/DNS/stats (the path that starts and ends in host memory, as
    pcap buffers do).  Reported in DESIGN.md; never the headline value."""
    n = len(offs) - 1
    pin_fr = N.PinnedBuffer(frames.nbytes)
    pin_fr.array[:] = frames
    pin_off = N.PinnedBuffer(offs.nbytes)
    pin_off.array[:] = offs.view(np.uint8)
    pin_out = N.PinnedBuffer(n * N.PKT_OUT_DTYPE.itemsize)
    pin_dns = N.PinnedBuffer(n * N.DNS_OUT_DTYPE.itemsize)
    st = np.zeros(1, dtype=N.STATS_DTYPE)
    no, nd = C.c_uint32(), C.c_uint32()

    def call():
        N.check(lib.fb_parse_classify(ctx, pin_fr.ptr, frames.nbytes, pin_off.ptr, n, pin_out.ptr, C.byref(no),
                                      pin_dns.ptr, C.byref(nd), None, st.ctypes.data, None))
    call()
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    el = time.perf_counter() - t0
    moved = frames.nbytes + offs.nbytes + no.value * N.PKT_OUT_DTYPE.itemsize + nd.value * N.DNS_OUT_DTYPE.itemsize
    for b in (pin_fr, pin_off, pin_out, pin_dns):
        b.free()
    return dict(value=round(calls * n / el / 1e6, 2), unit="Mpackets/s", ms_per_call=round(el * 1e3 / calls, 3),
                pcie_bytes_per_call=int(moved), pcie_GBs=round(moved * calls / el / 1e9, 2),
                note="synchronous fb_parse_classify on pinned host buffers (H2D + kernel + D2H, no overlap)")


def host_ring(N, lib, ctx, frames, offs, batches=16, slots=4, copy_threads=8):
    """The host ingest ring (fb_ring_*): pinned batches, H2D on a copy
    stream overlapping the previous batch's parse + session-table upsert, only the batch stats
    (and DNS side records) back -- the session table stays in HBM.  Two producers:
      copy:     fb_ring_push_block from ordinary (pageable) memory, one host thread (the memcpy
                into the pinned batch is the capture thread's copy, like the reference's to_vec);
      copy_mt:  the same with the block's copy split over `copy_threads` threads
                (fb_ring_config.copy_threads);
      per_frame: fb_ring_push once per frame from a native loop (the reference's reader thread hands
                over one frame per next_packet(), src/capture.rs:1088-1092);
      in_place: fb_ring_reserve_block with the frames already in the pinned batch (a capture
                engine writing into the ring; the offsets are still written per batch).
    Reported in DESIGN.md; never the headline value."""
    n = len(offs) - 1
    out = {}
    for name, threads in (("copy", 1), ("copy_mt", copy_threads)):
        if name == "copy_mt":
            out.update(_host_ring_runs(N, lib, ctx, frames, offs, batches, slots, threads, ("copy",),
                                       rename={"copy": "copy_mt"}))
            out["copy_mt"]["threads"] = threads
        else:
            out.update(_host_ring_runs(N, lib, ctx, frames, offs, batches, slots, threads,
                                       ("copy", "per_frame", "in_place")))
    return dict(unit="Mpackets/s", slots=slots, batch_frames=n, **out,
                note="fb_ring: pinned %d-batch ring, H2D (copy stream) + parse + session-table upsert "
                     "(compute stream) + stats D2H per batch, table kept in HBM" % slots)


def _host_ring_runs(N, lib, ctx, frames, offs, batches, slots, threads, modes, rename=None):
    n = len(offs) - 1
    cfg = N.FbRingConfig(slots, n, frames.nbytes, 0, threads)
    r = lib.fb_ring_create(ctx, C.byref(cfg))
    if not r:
        raise RuntimeError(lib.fb_last_error().decode())
    r = C.c_void_p(r)
    out = {}
    hb = C.CDLL(os.path.join(N.PKG, "libfb_hostbench.so"))
    hb.fb_hostbench_push_frames.restype = C.c_int
    hb.fb_hostbench_push_frames.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                            C.POINTER(C.c_double)]
    push_fn = C.cast(lib.fb_ring_push, C.c_void_p)
    try:
        N.check(lib.fb_flow_clear(ctx, None))
        rel = np.ascontiguousarray(offs[:-1], dtype=np.uint32)

        def copy_batch():
            N.check(lib.fb_ring_push_block(r, N.ptr(frames), N.ptr(offs), n))

        def in_place_batch(first):
            po, base = C.c_void_p(), C.c_uint32()
            p = lib.fb_ring_reserve_block(r, n, frames.nbytes, C.byref(po), C.byref(base))
            if not p:
                raise RuntimeError(lib.fb_last_error().decode())
            if first:  # the frames are written once per pinned slot, then stay in place
                C.memmove(p, frames.ctypes.data, frames.nbytes)
            o = np.ctypeslib.as_array((C.c_uint32 * n).from_address(po.value))
            np.add(rel, np.uint32(base.value), out=o)

        def per_frame_batches(k):
            sec = C.c_double()
            N.check(hb.fb_hostbench_push_frames(push_fn, r, N.ptr(frames), N.ptr(offs), n, k, C.byref(sec)))

        fns = {"copy": lambda i: copy_batch(), "in_place": lambda i: in_place_batch(i < slots)}
        for name in modes:
            if name == "per_frame":  # one native call per frame, `batches` batches' worth
                per_frame_batches(slots)  # warm-up
                N.check(lib.fb_ring_sync(r))
                t0 = time.perf_counter()
                per_frame_batches(batches)
                N.check(lib.fb_ring_sync(r))
                el = time.perf_counter() - t0
            else:
                fn = fns[name]
                for i in range(slots):  # warm-up: fill every slot once
                    fn(i)
                N.check(lib.fb_ring_sync(r))
                t0 = time.perf_counter()
                for i in range(batches):
                    fn(slots + i)
                N.check(lib.fb_ring_sync(r))
                el = time.perf_counter() - t0
            out[(rename or {}).get(name, name)] = dict(
                value=round(batches * n / el / 1e6, 2), ms_per_batch=round(el * 1e3 / batches, 3),
                pcie_GBs=round(batches * (frames.nbytes + offs.nbytes) / el / 1e9, 2))
        tot = np.zeros(1, dtype=N.STATS_DTYPE)
        nb = C.c_uint64()
        N.check(lib.fb_ring_stats(r, N.ptr(tot), C.byref(nb), None))
        if int(tot[0]["error"]) or int(tot[0]["n_session"]) + int(tot[0]["n_dns"]) + int(tot[0]["n_drop"]) != \
                int(nb.value) * n:
            raise RuntimeError("ring totals inconsistent: %s" % tot)
    finally:
        lib.fb_ring_destroy(r)
        lib.fb_flow_clear(ctx, None)
    return out


def c5_conservation(merged, records, local_flows, global_flows, unique_keys):
    """Invariants of the merged global session table (C5), whatever the exchange did: every SESSION
    record the ranks' parses emitted is counted exactly once -- the table's packets (orig + resp),
    payload bytes (outbound + inbound) and IP bytes (orig_ip + resp_ip) equal the sums over every
    rank's records --, the global flows lie between the largest rank table and the sum of all of
    them, and no key appears twice.  `merged` / `records`: dicts of packets, payload_bytes, ip_bytes.
    Raises RuntimeError naming every violated invariant; returns the checked values."""
    bad = []
    for k in ("packets", "payload_bytes", "ip_bytes"):
        if int(merged[k]) != int(records[k]):
            bad.append("%s: table %d != records %d" % (k, int(merged[k]), int(records[k])))
    if not (max(local_flows) <= global_flows <= sum(local_flows)):
        bad.append("global flows %d outside [max %d, sum %d] of the rank tables"
                   % (global_flows, max(local_flows), sum(local_flows)))
    if unique_keys != global_flows:
        bad.append("%d distinct keys in %d merged records" % (unique_keys, global_flows))
    if bad:
        raise RuntimeError("C5 conservation violated: " + "; ".join(bad))
    return dict(packets=int(merged["packets"]), payload_bytes=int(merged["payload_bytes"]),
                ip_bytes=int(merged["ip_bytes"]), local_flows=[int(x) for x in local_flows], unique_keys=unique_keys)


def c5_routed(N, lib, device, gpu_index, frames, offs, shard_first, global_n, world, dist, group, merged):
    """The routed global table (flodbadd_amd.distributed.RoutedSessionTable: every record to its key's
    owner before the update) over the same shard on a fresh context: its per-batch route / all_to_all /
    owner-update times, and its gathered table, which must equal the merged table of the export /
    merge path byte for byte (two independent constructions of the one global table; a difference
    raises and fails the run)."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.distributed import RoutedSessionTable, sort_by_ord
    from flodbadd_amd.sessions import SessionFilter
    n = len(offs) - 1
    cap = FlodbaddGpuCapture(gpu_index, session_filter=SessionFilter.GlobalOnly, flow_capacity=1 << 21,
                             max_batch_packets=n, grow=False)
    try:
        rt = RoutedSessionTable(dist, cap, group=group, device=device)
        rt.process(frames, offs, shard_first, global_n)  # warm-up (communicators, scratch)
        cap.clear_all_sessions()
        dist.barrier(group=group)
        timing = {}
        t0 = time.perf_counter()
        rt.process(frames, offs, shard_first, global_n, timing=timing)
        dist.barrier(group=group)
        el = time.perf_counter() - t0
        table = rt.global_table()
    finally:
        cap.close()
    m = np.ascontiguousarray(merged.cpu().numpy()).view(N.FLOW_REC_DTYPE).reshape(-1)
    a, b = sort_by_ord(table.copy()), sort_by_ord(m.copy())
    a["slot"] = 0
    b["slot"] = 0
    if len(a) != len(b) or a.tobytes() != b.tobytes():
        raise RuntimeError("routed global table (%d flows) differs from the merged one (%d flows)" % (len(a), len(b)))
    return dict(batch_ms=round(el * 1e3, 3), Mpackets_s=round(global_n / el / 1e6, 1),
                stages_ms={k: round(v, 3) for k, v in timing.items() if k.endswith("_ms")},
                records_sent_to_other_ranks=int(timing.get("records_out", 0)), equals_merged_table=True,
                note="per global batch: parse + route (fb_route_records_dev), all_to_all of the records, the "
                     "owner's update (fb_flow_update_records_dev); gathered table == the export/merge path's")


def c5_flow_reduce(N, lib, ctx, per_rank, rank, world, dist, group, device):
    """BASELINE config C5 after the timed region: rank r's shard of a world x per_rank frame batch
    (C4 mix, flow pool 2^20; packets [r * per_rank, (r+1) * per_rank)) through the fused parse +
    classify + session-table kernels, then the global session table (flodbadd_amd.distributed:
    owner-grouped export and owner merge in the library, all_to_all + all_gather over RCCL)."""
    from flodbadd_amd import synth
    from flodbadd_amd.distributed import global_flow_table
    shard_first = rank * per_rank
    frames, offs = synth.generate(4, per_rank, first=shard_first)
    n = len(offs) - 1
    N.check(lib.fb_flow_clear(ctx, None))
    d_fr = N.DeviceBuffer(frames.nbytes).upload(frames)
    d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
    d_out = N.DeviceBuffer(n * N.PKT_OUT_DTYPE.itemsize)
    d_st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
    ev0, ev1 = N.Event(), N.Event()
    # once untimed (grows the context's update scratch to the shard), then the timed update
    N.check(lib.fb_process_dev(ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, None, None, d_st.ptr, None))
    N.check(lib.fb_flow_clear(ctx, None))
    ev0.record(None)
    N.check(lib.fb_process_dev(ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, None, None, d_st.ptr, None))
    ev1.record(None)
    flow_ms = ev0.elapsed_ms(ev1)
    cnt = C.c_uint64()
    N.check(lib.fb_flow_count(ctx, C.byref(cnt), None))
    # what this rank's parse emitted (the records the table must account for, exactly once)
    st = d_st.download(np.zeros(1, dtype=N.STATS_DTYPE))
    ns = int(st[0]["n_session"])
    recs = d_out.download(np.zeros(max(ns, 1), dtype=N.PKT_OUT_DTYPE))[:ns]
    rec_sums = [ns, int(recs["packet_length"].sum(dtype=np.uint64)), int(recs["ip_packet_length"].sum(dtype=np.uint64))]
    del recs

    def export_merge(timing=None):
        # the library exports the owner groups into a device tensor, the collectives move them
        # (RCCL with device tensors; gloo via host memory), the library merges each owner's records
        merged = global_flow_table(dist, ctx, shard_first=shard_first, device=device, group=group, as_tensor=True,
                                   timing=timing)
        if device.type == "cuda":
            import torch
            torch.cuda.synchronize(device)
        return int(cnt.value), merged

    # the first merge also sets up the group's communicators and loads the sort kernels: timed apart
    t0 = time.perf_counter()
    export_merge()
    first = time.perf_counter() - t0
    t0 = time.perf_counter()
    local, merged = export_merge()
    el = time.perf_counter() - t0
    # a third pass with every stage drained and timed apart: the collectives' time and bytes beside the
    # library's export and merge kernels
    stages = {}
    export_merge(stages)
    for b in (d_fr, d_off, d_out, d_st):
        b.free()
    import torch
    t = np.array([flow_ms], dtype=np.float64)
    if world > 1:  # the slowest rank's update: the aggregate rate of the concurrent shards
        tt = torch.tensor(t, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        t = tt.cpu().numpy()
    # conservation of the merged table against every rank's records (a violation fails the run)
    rs = torch.tensor(rec_sums, dtype=torch.int64, device=device)
    lf = torch.tensor([local], dtype=torch.int64, device=device)
    lfs = [torch.zeros_like(lf) for _ in range(world)]
    if world > 1:
        dist.all_reduce(rs, group=group)
        dist.all_gather(lfs, lf, group=group)
    else:
        lfs = [lf]
    cols = merged[:, 5:11].sum(dim=0).tolist() if len(merged) else [0] * 6  # fb_flow_rec counters
    uniq = int(torch.unique(merged[:, :5], dim=0).shape[0]) if len(merged) else 0
    rs = rs.tolist()
    cdev = C.c_int(0)
    N.check(lib.fb_ctx_device(ctx, C.byref(cdev)))
    routed = c5_routed(N, lib, device, cdev.value, frames, offs, shard_first, n * world, world, dist, group, merged)
    conserved = c5_conservation(
        dict(packets=cols[2] + cols[3], payload_bytes=cols[0] + cols[1], ip_bytes=cols[4] + cols[5]),
        dict(packets=rs[0], payload_bytes=rs[1], ip_bytes=rs[2]),
        [int(x.item()) for x in lfs], int(len(merged)), uniq)
    return dict(ranks_in_group=dist.get_world_size(group), frames_per_rank=n, total_frames=n * world,
                conservation=conserved, routed=routed,
                local_flows=local, global_flows=int(len(merged)),
                flow_update_ms=round(flow_ms, 3), update_Mpackets_s=round(world * n / float(t[0]) / 1e3, 1),
                export_merge_ms=round(el * 1e3, 3), export_merge_first_call_ms=round(first * 1e3, 3),
                stages_ms={k: round(v, 3) for k, v in stages.items() if k.endswith("_ms")},
                collective_bytes={k: int(v) for k, v in stages.items() if k.endswith("_bytes")},
                collective_GBs=round((stages.get("a2a_bytes", 0) + stages.get("gather_bytes", 0)) /
                                     max(stages.get("a2a_ms", 0) + stages.get("gather_ms", 0), 1e-9) / 1e6, 2),
                note="per-rank fused parse+flow upsert of the rank's shard, then the global session table: "
                     "fb_flow_export_merge_dev (owner groups, device tensor), all_to_all to the owners, "
                     "fb_flow_merge_dev on each owner, all_gather of the merged records (left on the device)")


def stream_copy(device, nbytes=1 << 30, reps=20):
    """the measured stream-copy bandwidth beside the 8 TB/s spec -- a 16-B-per-lane
    copy kernel (libfb_bwref.so, fb_bwref.hip) over `nbytes` (well past the 256 MB Infinity Cache),
    timed with events on the stream it runs on; read + written bytes / time.
    `roofline.frac_of_copy` relates the dominant kernel to what a plain copy reaches on the same GPU
    (a reference point, not the product path; hipMemcpyAsync device to device reached only
    ~4.7 TB/s, so it is not the yardstick)."""
    from flodbadd_amd import _native as N
    lib = C.CDLL(os.path.join(N.PKG, "libfb_bwref.so"))
    lib.fb_bwref_copy.restype = C.c_int
    lib.fb_bwref_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_float)]
    N.check(N.gpu_lib().fb_set_device(device))
    src, dst = N.DeviceBuffer(nbytes), N.DeviceBuffer(nbytes)
    ms = C.c_float()
    rc = lib.fb_bwref_copy(dst.ptr, src.ptr, nbytes, reps, C.byref(ms))
    del src, dst
    if rc != 0:
        raise RuntimeError("fb_bwref_copy failed: %d" % rc)
    return round(2.0 * nbytes * reps / (ms.value / 1e3) / 1e9, 1)


def usable_cores():
    """Host cores this process may use: the CPU affinity set, capped by the cgroup CPU quota (the
    GPU box's CPU share) and by OMP_NUM_THREADS when the harness sets it to that share.  Returns
    (cores, how it was decided)."""
    aff = len(os.sched_getaffinity(0))
    n, why = aff, "sched_getaffinity %d" % aff
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
            why += ", cgroup cpu.max quota %d" % quota
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < n:
        why += ", OMP_NUM_THREADS %s (the box's CPU share for one GPU)" % omp
        n = int(omp)
    return n, why


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        return ""


def _timed_passes(fn, budget):
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget:
            return passes, el


def cpu_baseline(frames, offs, seconds):
    """The oracle (C restatement of src/packets.rs parse + classify) on the same batch, repeated
    for about `seconds` of wall time: a bounded sample of the same workload.  SURVEY.md 8d asks for
    (i) one thread, like the reference's one processor task per interface (src/capture.rs:1027),
    and (ii) all host cores: the main object is (ii) (orc_parse_classify_mt, contiguous ranges in
    parallel, compacted in packet order; `cores` = usable_cores()), with (i) beside it."""
    from oracle import coracle
    cfg = coracle.make_cfg(1)  # FlodbaddCapture::new() default filter: GlobalOnly
    n = len(offs) - 1
    out = np.zeros(n, dtype=coracle.PKT_OUT_DTYPE)
    dns = np.zeros(n, dtype=coracle.DNS_OUT_DTYPE)
    st = np.zeros(1, dtype=coracle.STATS_DTYPE)
    no, nd = C.c_uint32(), C.c_uint32()
    L = coracle.lib()
    threads, why = usable_cores()

    def run(t):
        if t == 1:
            L.orc_parse_classify(C.byref(cfg), frames.ctypes.data, frames.nbytes, offs.ctypes.data, n,
                                 out.ctypes.data, C.byref(no), dns.ctypes.data, C.byref(nd), None, st.ctypes.data)
        else:
            L.orc_parse_classify_mt(C.byref(cfg), frames.ctypes.data, frames.nbytes, offs.ctypes.data, n,
                                    out.ctypes.data, C.byref(no), dns.ctypes.data, C.byref(nd), st.ctypes.data, t)
    p1, e1 = _timed_passes(lambda: run(1), seconds / 2)
    pm, em = _timed_passes(lambda: run(threads), seconds / 2)
    return dict(value=round(pm * n / em / 1e6, 3), unit="Mpackets/s", cores=threads, kind="port",
                cores_rule=why,
                sample="%d passes over the %d-frame batch (%.1f s, %d threads, C restatement oracle/oracle.c, %s)"
                       % (pm, n, em, threads, _cpu_model()),
                single_thread=dict(value=round(p1 * n / e1 / 1e6, 3), cores=1,
                                   sample="%d passes (%.1f s, 1 thread)" % (p1, e1)))


def cpu_baseline_c4(frames, offs, seconds):
    """C4 CPU baseline: parse + classify + the session-table upsert (orc_pipeline_mt: ranges
    parsed in parallel, then every thread upserts the keys it owns, in packet order, into its own
    table; orc_pipeline for one thread) on a bounded sample: the first 2M frames of the C4 batch,
    each pass into fresh tables (the GPU's timed steps update a warm table: the CPU passes after
    the first do the same, tables are cleared only between the two thread counts)."""
    from oracle import coracle
    cfg = coracle.make_cfg(1)
    m = min(len(offs) - 1, 1 << 21)
    o = np.ascontiguousarray(offs[: m + 1])
    threads, why = usable_cores()
    L = coracle.lib()
    scratch = np.zeros(m, dtype=coracle.PKT_OUT_DTYPE)
    st = np.zeros(1, dtype=coracle.STATS_DTYPE)
    one = coracle.Flows()
    p1, e1 = _timed_passes(lambda: L.orc_pipeline(C.byref(cfg), one.h, frames.ctypes.data, frames.nbytes,
                                                  o.ctypes.data, m, scratch.ctypes.data, st.ctypes.data), seconds / 2)
    tabs = [coracle.Flows() for _ in range(threads)]
    pm, em = _timed_passes(lambda: coracle.pipeline_mt(cfg, frames, o, threads, tabs), seconds / 2)
    return dict(value=round(pm * m / em / 1e6, 3), unit="Mpackets/s", cores=threads, kind="port", cores_rule=why,
                sample="%d passes over the first %d frames of the C4 batch, parse + classify + session upsert "
                       "(%.1f s, %d threads, oracle/oracle.c orc_pipeline_mt, %s)" % (pm, m, em, threads, _cpu_model()),
                single_thread=dict(value=round(p1 * m / e1 / 1e6, 3), cores=1,
                                   sample="%d passes (%.1f s, 1 thread, orc_pipeline)" % (p1, e1)))


def load_traffic(config_id, bpl=1):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (tools/prof_summary.py: separate FETCH_SIZE / WRITE_SIZE passes, FETCH x2 for gfx950), scaled to
    `bpl` batches per launch, and the tag of the profiled run it comes from."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f).get(str(config_id), {})
        b = d.get("hbm_bytes_per_launch")
        return (None if b is None else b / d.get("batches_per_launch", 1) * bpl), d.get("tag")
    except (OSError, ValueError):
        return None, None


def c4_split(N, lib, ctx, main_r, n, steps, warmup, rank, world, dist, mode, pipe, synth_kw=None, records=True):
    """The C4 step's parse / update split: for the pipelined line a one-stream fb_process_seg_dev run
    (fewer steps) whose stage event splits each step; plus the side timings the C4 main run took
    (history, enrichment, DNS parse)."""
    extra = {}
    sg = main_r["stage"]
    split = sg
    if pipe:  # the stage split and the one-stream rate from fb_process_seg_dev, fewer steps
        st_s = max(steps // 2, 10)
        rs = run_config(N, lib, ctx, 4, n, st_s, max(warmup // 2, 2), 1, rank, world, dist, flow=True,
                        mode=mode, synth_kw=synth_kw, stage_extras=False, records=records)
        split = rs["stage"]
        extra["c4_sync"] = dict(value=round(world * n * st_s / rs["elapsed"] / 1e6, 2), unit="Mpackets/s",
                                ms_per_step=round(rs["elapsed"] * 1e3 / st_s, 4),
                                note="fb_process_seg_dev: parse then update on one stream, no overlap")
    extra["c4_stages"] = dict(parse_ms=round(split["parse_ms"], 4), flow_update_ms=round(split["flow_ms"], 4),
                              stages_note="split by the stage event fb_process%s_dev records between its "
                                          "parse and its update%s" % ("_seg" if mode == "seg" else "",
                                                                      " (one-stream run)" if pipe else ""),
                              history_ms=round(sg["history_ms"], 4), history_chars=sg["history_chars"],
                              enrich_ms=sg["enrich_ms"], enrich_Mflows_s=sg["enrich_Mflows_s"],
                              enrich_tables=sg["enrich_tables"],
                              dns_parse_ms=sg["dns_parse_ms"], dns_Mmsgs_s=sg["dns_Mmsgs_s"],
                              dns_payload_GBs=sg["dns_payload_GBs"], dns_ok=sg["dns_ok"],
                              dns_workload="1M port-53 payloads (synth.dns_workload), device-resident",
                              flows_in_table=sg["flows"],
                              parse_GBs=round(main_r["algo_bytes"] / split["parse_ms"] / 1e6, 1),
                              flow_Mrec_s=round(main_r["stats"]["n_session"] / split["flow_ms"] / 1e3, 1))
    return extra


def c4_algo_bytes(r, records=True):
    """Algorithmic bytes of one C4 step: the parse's (header windows, offsets,
    records written -- none when the table is the only output) + the update's: every SESSION record
    read once (56 B; table-only: nothing, the table is built from the headers) and every flow's
    128-B table slot read and written once."""
    return r["algo_bytes"] + (56 * r["stats"]["n_session"] if records else 0) + 2 * 128 * r["stage"]["flows"]


def c4_line(N, lib, ctx, steps, warmup, rank, world, dist, cpu_seconds):
    """BASELINE configs[3] (C4) as an extra of the default run, so the driver times it: 10,485,760
    IMIX frames per step through the pipelined fused call (fb_process_seg_async_dev, two rotating
    buffer sets, joined inside the timed region), its parse / update split, the step's algorithmic
    bytes against HBM peak, and the CPU parse + upsert baseline beside it."""
    n = 10 * (1 << 20)
    # the reference's capture loop keeps only the session table (each ParsedPacket is dropped after
    # process_parsed_packet, src/capture.rs:1036-1061): the line's fused calls do the same
    # (fb_set_session_records 0); c4_records times them storing every SESSION record too
    r = run_config(N, lib, ctx, 4, n, steps, warmup, 2, rank, world, dist, flow=True, mode="seg", pipelined=True,
                   records=False)
    out = dict(value=round(world * n * steps / r["elapsed"] / 1e6, 2), unit="Mpackets/s",
               ms_per_step=round(r["elapsed"] * 1e3 / steps, 4), steps=steps, warmup=warmup,
               workload=WORKLOADS[4], output="fb_process_seg_async_dev (pipelined parse + session upsert; the "
                                             "session table and the DNS side records are the output)")
    ach = c4_algo_bytes(r, records=False) * steps / (r["ev_ms"] / 1e3) / 1e9
    out["roofline"] = dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                           frac=round(ach / HBM_PEAK_GBS, 4), algo_bytes_per_step=int(c4_algo_bytes(r, records=False)),
                           note="whole step (parse + update, overlapped) over its algorithmic bytes")
    rr = run_config(N, lib, ctx, 4, n, steps, warmup, 2, rank, world, dist, flow=True, mode="seg", pipelined=True,
                    stage_extras=False)
    out["c4_records"] = dict(value=round(world * n * steps / rr["elapsed"] / 1e6, 2), unit="Mpackets/s",
                             ms_per_step=round(rr["elapsed"] * 1e3 / steps, 4),
                             note="the same pipelined calls also storing every SESSION record (fb_pkt_out) in d_out")
    out.update(c4_split(N, lib, ctx, r, n, steps, warmup, rank, world, dist, "seg", True, records=False))
    # C4 also with Zipf(1.1) flow popularity -- the same pipelined table-only calls
    rz = run_config(N, lib, ctx, 4, n, steps, warmup, 2, rank, world, dist, flow=True, mode="seg", pipelined=True,
                    records=False, synth_kw=dict(zipf=1, zipf_s=1.1), stage_extras=False)
    out["c4_zipf"] = dict(value=round(world * n * steps / rz["elapsed"] / 1e6, 2), unit="Mpackets/s",
                          ms_per_step=round(rz["elapsed"] * 1e3 / steps, 4), steps=steps,
                          note="Zipf(1.1) flow popularity over the 2^20 pool, otherwise as the C4 line")
    # the batch a capture loop flushing every ~1 ms hands over: 1,048,576 frames per fused call
    m, s1 = 1 << 20, max(steps * 5, 100)
    r1 = run_config(N, lib, ctx, 4, m, s1, warmup * 2, 2, rank, world, dist, flow=True, mode="seg", pipelined=True,
                    records=False, stage_extras=False)
    out["c4_1m"] = dict(value=round(world * m * s1 / r1["elapsed"] / 1e6, 2), unit="Mpackets/s",
                        ms_per_call=round(r1["elapsed"] * 1e3 / s1, 4), steps=s1, frames_per_call=m,
                        note="the C4 mix in 1M-frame fb_process_seg_async_dev calls (table-only, pipelined)")
    # the same C4 line on a timed context (capture timestamps: the 5-s segment timeout and the capture
    # times per flow, fb_time.hip) -- its own context, the table's time plane beside it
    tcfg = N.FbConfig()
    tcfg.abi_version = N.FB_ABI_VERSION
    tcfg.filter = N.FB_FILTER_GLOBAL_ONLY
    tcfg.max_batch_packets = n
    tcfg.flow_capacity = 1 << 21
    tcfg.flags = N.FB_CFG_FIXED_TABLE | N.FB_CFG_TIMED
    cdev = C.c_int(0)
    N.check(lib.fb_ctx_device(ctx, C.byref(cdev)))
    tctx = lib.fb_create(cdev.value, C.byref(tcfg))
    if tctx:
        tctx = C.c_void_p(tctx)
        try:
            rt = run_config(N, lib, tctx, 4, n, steps, warmup, 2, rank, world, dist, flow=True, mode="seg",
                            pipelined=True, records=False, stage_extras=False, timed=True)
            out["c4_timed"] = dict(value=round(world * n * steps / rt["elapsed"] / 1e6, 2), unit="Mpackets/s",
                                   ms_per_step=round(rt["elapsed"] * 1e3 / steps, 4), steps=steps,
                                   note="the C4 line on a timed context (FB_CFG_TIMED): per-frame capture times, "
                                        "the capture-time pass after each update")
        finally:
            lib.fb_destroy(tctx)
    else:
        out["c4_timed"] = {"error": lib.fb_last_error().decode()[:200]}
    if rank == 0 and world == 1 and cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline_c4(r["frames"], r["offs"], cpu_seconds)
    return out


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N child processes of this script, rank r with
    RANK = LOCAL_RANK = r, WORLD_SIZE = N and a loopback rendezvous (torchrun's environment), and
    wait for all of them.  The parent never touches the GPU and never execs (it runs the children
    as subprocesses); rank 0 prints the JSON line.  Returns the exit status: 0 only if every rank
    exited 0 (a failing rank ends the others)."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                for q in live:  # a rank died: the others would wait for it at the next collective
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return status


_result_out = None  # the process's original stdout: only the result line goes there (_emit)


def _quiet_stdout():
    """Send fd 1 to stderr for the rest of the run, keeping the original stdout for the one result
    line: libraries write their notices to fd 1 from native code (gloo's "Rank r is connected to
    ... peer ranks", RCCL banners), which would otherwise land before the JSON line."""
    global _result_out
    sys.stdout.flush()
    _result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def _emit(obj):
    out = _result_out or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def c5_checked(run, world, gpus, dist):
    """Run the C5 exchange (`run()` -> its extra dict) on every rank of a world > 1 and agree on the
    outcome: an exception, or a group that does not hold --gpus ranks, fails it.  Every rank then
    learns over the default group whether all succeeded (a rank whose peer failed inside a collective
    leaves it by the C5 group's timeout).  Returns (extra dict, ok on every rank)."""
    import torch
    try:
        res = run()
        ok = res.get("ranks_in_group") == gpus
        if not ok:
            res["error"] = "the C5 group holds %s ranks, --gpus %d" % (res.get("ranks_in_group"), gpus)
    except Exception as e:
        res, ok = {"error": repr(e)[:300]}, False
    t = torch.tensor([0 if ok else 1], dtype=torch.int64)
    flags = [t]
    if world > 1:
        flags = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(flags, t)
    failed = [r for r, f in enumerate(flags) if int(f[0])]
    if failed:
        res["failed_ranks"] = failed
        res.setdefault("error", "the C5 exchange failed on rank(s) %s" % failed)
    return res, not failed


def world_check(args, world, rank):
    """--world-check: the launch plumbing only (no GPU): every rank joins the gloo group, the ranks
    all-reduce their rank numbers, rank 0 prints what the group saw."""
    import torch
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
    t = torch.tensor([rank, 1], dtype=torch.int64)
    if world > 1:
        tdist.all_reduce(t)
    line = {"n_gpus": world, "requested_gpus": args.gpus, "group_size": int(t[1]),
            "rank_sum": int(t[0]), "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT"))}
    c5_ok = True
    if world > 1:
        # the C5 outcome plumbing with a stand-in exchange (FB_C5_INJECT=fail: rank 1 raises;
        # =group: the group reports fewer ranks than --gpus; =conservation: every rank's merged
        # table fails c5_conservation)
        inject = os.environ.get("FB_C5_INJECT", "")

        def run():
            if inject == "fail" and rank == 1:
                raise RuntimeError("injected C5 merge failure")
            if inject == "conservation":  # a merged table that lost one packet's bytes
                sums = dict(packets=1000, payload_bytes=64000, ip_bytes=104000)
                c5_conservation(dict(sums, payload_bytes=63990), sums, [600, 500], 900, 900)
            return {"ranks_in_group": world - 1 if inject == "group" else tdist.get_world_size()}
        res, c5_ok = c5_checked(run, world, args.gpus, tdist)
        line["extra"] = {"c5_flow_reduce": res}
        line["c5_ok"] = c5_ok
    if rank == 0:
        _emit(line)
    if world > 1:
        tdist.destroy_process_group()
    if not c5_ok:
        raise SystemExit("C5 exchange failed on some rank")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--packets", type=int, default=None, help="frames per GPU per step")
    ap.add_argument("--rotate", type=int, default=None, help="distinct device batches cycled")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-imix", action="store_true", help="skip the secondary IMIX (C3) measurement")
    ap.add_argument("--no-c4", action="store_true", help="config 2: skip the C4 (parse + session table) extra")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (pinned H2D/D2H) measurement")
    ap.add_argument("--no-flow-reduce", action="store_true", help="N>1: skip the C5 global flow-counter exchange")
    ap.add_argument("--c5-frames", type=int, default=10 * (1 << 20),
                    help="N>1: frames per rank of the C5 shard (BASELINE configs[4]: 80M over 8 GPUs)")
    ap.add_argument("--mode", choices=["seg", "dense"], default="seg",
                    help="output layout: per-wavefront segments (default) or one batch-wide compaction")
    ap.add_argument("--no-other-mode", action="store_true", help="skip timing the other output layout")
    ap.add_argument("--no-single-launch", action="store_true", help="skip timing one batch per launch")
    ap.add_argument("--no-queue", action="store_true", help="skip timing one batch per call through fb_seg_queue")
    ap.add_argument("--no-copy-ref", action="store_true", help="skip the stream-copy bandwidth reference")
    ap.add_argument("--batches-per-launch", type=int, default=None,
                    help="seg mode: batches (steps) per kernel launch (fb_parse_classify_seg_batches_dev); "
                         "default = the rotated batches (C2 / C3 32), 1 for C4")
    ap.add_argument("--c4-sync", action="store_true",
                    help="C4: time fb_process_seg_dev (one stream) instead of the pipelined fb_process_seg_async_dev")
    ap.add_argument("--table-only", action="store_true",
                    help="C4 (seg): the fused calls keep only the session table (fb_set_session_records 0)")
    ap.add_argument("--zipf", type=float, default=None,
                    help="profiling: the main run with Zipf(s) flow popularity instead of uniform")
    ap.add_argument("--world-check", action="store_true",
                    help="launch plumbing only: the ranks join the group and rank 0 reports it (no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process only starts the N ranks (before any HIP call) and waits
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but the launcher started %d ranks" % (args.gpus, world))
    _quiet_stdout()
    if args.world_check:
        return world_check(args, world, rank)
    dist = None
    if world > 1:
        # (torch is imported before the library initialises HIP: imported after it, torch saw no GPU
        # on the box -- tools/experiments/torch_after_lib.py -- and the C5 exchange needs its tensors)
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist

    from flodbadd_amd import _native as N
    lib = N.gpu_lib()
    ndev = N.device_count()
    if ndev == 0:
        raise SystemExit("no HIP device visible")
    device = local % ndev
    cfg = N.FbConfig()
    cfg.abi_version = N.FB_ABI_VERSION
    cfg.filter = N.FB_FILTER_GLOBAL_ONLY  # FlodbaddCapture::new() default (src/capture.rs:108)
    cfg.max_batch_packets = 1 << 24
    cfg.flow_capacity = 1 << 21  # C5 exchange: the rank's shard flows (<= 2^20 in the C4/C5 pool)
    cfg.flags = N.FB_CFG_FIXED_TABLE  # sized for the pool (1.45M flows): no growth mid-run
    N.check(lib.fb_set_device(device))
    ctx = lib.fb_create(device, C.byref(cfg))
    if not ctx:
        raise SystemExit("fb_create failed: %s" % lib.fb_last_error().decode())
    ctx = C.c_void_p(ctx)

    n = args.packets or (10 * (1 << 20) if args.config == 4 else 1 << 20)
    # C2 / C3: 32 distinct batches (4 / 12 GB, far past the 256 MB Infinity Cache), so any K <= 32
    # steps is one launch and longer runs are near-equal launches of up to 32 batches (plan_launches)
    # C4 (segmented): the pipelined fused call, each batch's table update overlapping the next
    # batch's parse, on two rotating buffer sets; --c4-sync times fb_process_seg_dev instead
    pipe = args.config == 4 and args.mode == "seg" and not args.c4_sync
    rotate = args.rotate or (32 if args.config in (2, 3) else (2 if pipe else 1))
    bpl = min(args.batches_per_launch or rotate, rotate, MAX_SEG_BATCHES) \
        if (args.mode == "seg" and args.config != 4) else 1
    main_kw = dict(zipf=1, zipf_s=args.zipf) if args.zipf else None
    main_r = run_config(N, lib, ctx, args.config, n, args.steps, args.warmup, rotate, rank, world, dist,
                        flow=args.config == 4, mode=args.mode, bpl=bpl,
                        synth_kw=main_kw, pipelined=pipe, records=not args.table_only)
    # the dominant kernel's launches: algorithmic bytes per launch / average launch duration
    per_launch_s = main_r["ev_ms"] / 1e3 / main_r["launches"]
    algo_per_launch = main_r["algo_bytes"] * args.steps / main_r["launches"]
    achieved = algo_per_launch / per_launch_s / 1e9
    value = world * n * args.steps / main_r["elapsed"] / 1e6
    per_rank = None
    if dist:  # every rank's own kernel rate (its GPU's roofline fraction) beside the aggregate
        import torch
        mine = torch.tensor([achieved, n * args.steps / main_r["local_elapsed"] / 1e6], dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [dict(rank=r, Mpackets_s=round(float(t[1]), 2), roofline_frac=round(float(t[0]) / HBM_PEAK_GBS, 4))
                    for r, t in enumerate(allr)]

    extra = {}
    if main_r["stage"]:
        extra.update(c4_split(N, lib, ctx, main_r, n, args.steps, args.warmup, rank, world, dist, args.mode, pipe,
                              main_kw, records=not args.table_only))
    if args.config == 4 and not args.no_other_mode:  # C4 also with Zipf(1.1) flow popularity
        rz = run_config(N, lib, ctx, 4, n, max(args.steps // 2, 5), max(args.warmup // 2, 2), rotate, rank, world,
                        dist, flow=True, mode=args.mode, synth_kw=dict(zipf=1, zipf_s=1.1))
        sz = rz["stage"]
        extra["c4_zipf"] = dict(value=round(world * n * max(args.steps // 2, 5) / rz["elapsed"] / 1e6, 2),
                                unit="Mpackets/s", parse_ms=round(sz["parse_ms"], 4),
                                flow_update_ms=round(sz["flow_ms"], 4), flows_in_table=sz["flows"],
                                history_ms=round(sz["history_ms"], 4))
    if bpl > 1 and not args.no_single_launch:  # the same workload with one batch per launch
        st_1 = max(args.steps // 2, 10)
        r1 = run_config(N, lib, ctx, args.config, n, st_1, max(args.warmup // 2, 2), rotate, rank, world, dist,
                        mode=args.mode, bpl=1)
        pl1 = r1["ev_ms"] / 1e3 / r1["launches"]
        extra["single_batch_launch"] = dict(value=round(world * n * st_1 / r1["elapsed"] / 1e6, 2),
                                            unit="Mpackets/s", ms_per_step=round(r1["elapsed"] * 1e3 / st_1, 4),
                                            roofline_achieved_GBs=round(r1["algo_bytes"] / pl1 / 1e9, 1),
                                            roofline_frac=round(r1["algo_bytes"] / pl1 / 1e9 / HBM_PEAK_GBS, 4))
        if not args.no_queue:  # one batch per call through the resident queue-fed kernel
            try:
                qr = queue_line(N, lib, ctx, args.config, n, max(args.steps, 512), max(args.warmup // 2, 8), rotate)
                qr["value"] = round(qr["value"] * world, 2)
                extra["single_batch_queue"] = qr
            except Exception as e:  # reported beside the line; the headline does not depend on it
                extra["single_batch_queue"] = {"error": repr(e)[:300]}
            if args.config == 2 and world == 1:
                try:
                    extra["single_batch_queue_table"] = queue_table_line(N, lib, ctx)
                except Exception as e:
                    extra["single_batch_queue_table"] = {"error": repr(e)[:300]}
    # N > 1: the scaling line needs only the headline path (the other layout is timed at N = 1)
    if not args.no_other_mode and world == 1:
        other = "dense" if args.mode == "seg" else "seg"
        st_o = max(args.steps // 2, 10)
        ro = run_config(N, lib, ctx, args.config, n, st_o, max(args.warmup // 2, 2), rotate, rank, world, dist,
                        flow=args.config == 4, mode=other)
        plo = ro["ev_ms"] / 1e3 / st_o
        extra["mode_" + other] = dict(value=round(world * n * st_o / ro["elapsed"] / 1e6, 2), unit="Mpackets/s",
                                      ms_per_step=round(ro["elapsed"] * 1e3 / st_o, 4),
                                      roofline_achieved_GBs=round(ro["algo_bytes"] / plo / 1e9, 1),
                                      roofline_frac=round(ro["algo_bytes"] / plo / 1e9 / HBM_PEAK_GBS, 4))
    if not args.no_imix and args.config == 2:
        steps3 = max(args.steps // 2, 10)
        bpl3 = 32 if args.mode == "seg" and bpl > 1 else 1
        r3 = run_config(N, lib, ctx, 3, 1 << 20, steps3, max(args.warmup // 2, 2), 32, rank, world, dist,
                        mode=args.mode, bpl=bpl3)
        pl3 = r3["ev_ms"] / 1e3 / r3["launches"]
        algo3 = r3["algo_bytes"] * steps3 / r3["launches"]
        extra["imix_c3"] = dict(value=round(world * (1 << 20) * steps3 / r3["elapsed"] / 1e6, 2),
                                unit="Mpackets/s", ms_per_step=round(r3["elapsed"] * 1e3 / steps3, 4),
                                roofline_achieved_GBs=round(algo3 / pl3 / 1e9, 1),
                                roofline_frac=round(algo3 / pl3 / 1e9 / HBM_PEAK_GBS, 4),
                                batches_per_launch=bpl3, algo_bytes_per_batch=r3["algo_bytes"])

    if args.config == 2 and not args.no_c4:  # BASELINE configs[3] in the default (driver-timed) run
        extra["c4"] = c4_line(N, lib, ctx, max(args.steps // 10, 20), 5, rank, world, dist,
                              0 if args.no_cpu_baseline else args.cpu_seconds / 2)
    if not args.no_host and rank == 0 and args.config == 2:
        extra["host_inclusive_c2"] = host_inclusive(N, lib, ctx, main_r["frames"], main_r["offs"])
        try:
            extra["host_ring_c2"] = host_ring(N, lib, ctx, main_r["frames"], main_r["offs"])
        except Exception as e:  # reported, never allowed to break the bench line
            extra["host_ring_c2"] = {"error": repr(e)[:300]}

    c5_ok = True
    if world > 1 and not args.no_flow_reduce:
        try:
            import torch
            import torch.distributed as tdist
            # RCCL over xGMI (one GPU per rank); FB_C5_BACKEND=gloo exercises the same exchange with
            # CPU tensors when the ranks share one GPU (rehearsal on a one-GPU box)
            backend = os.environ.get("FB_C5_BACKEND", "nccl")
            dev = torch.device("cuda", device) if backend == "nccl" else torch.device("cpu")
            torch.cuda.set_device(torch.device("cuda", device))  # the library's exports land on this GPU
            import datetime
            g = tdist.new_group(backend=backend, timeout=datetime.timedelta(seconds=180))
        except Exception as e:
            g, setup_error = None, repr(e)[:300]

        def run():
            if g is None:
                raise RuntimeError("C5 group setup failed: %s" % setup_error)
            r = c5_flow_reduce(N, lib, ctx, args.c5_frames, rank, world, tdist, g, dev)
            r["backend"] = "rccl" if backend == "nccl" else backend
            return r
        # a failed exchange or a short group fails the run (non-zero exit after the line is printed)
        extra["c5_flow_reduce"], c5_ok = c5_checked(run, world, args.gpus, dist)

    copy_gbs = None
    if rank == 0 and not args.no_copy_ref:  # (after the timed region)
        try:
            copy_gbs = stream_copy(device)
        except Exception as e:  # a reference point: reported, never allowed to break the bench line
            print("stream copy reference failed: %r" % (e,), file=sys.stderr)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(main_r["frames"], main_r["offs"], args.cpu_seconds)

    lib.fb_destroy(ctx)
    if bpl > 1:
        output_desc = ("per-64-frame wavefront-compacted segments (fb_parse_classify_seg_batches_dev: "
                       "up to %d batches per launch, each with its own outputs and stats)" % bpl)
    elif args.mode == "seg" and args.config == 4:
        output_desc = ("per-64-frame wavefront-compacted segments + session-table upsert " +
                       ("(fb_process_seg_async_dev: each batch's update overlaps the next batch's parse, "
                        "2 rotating buffer sets)" if pipe else "(fb_process_seg_dev)"))
    elif args.mode == "seg":
        output_desc = "per-64-frame wavefront-compacted segments (fb_parse_classify_seg_dev)"
    else:
        output_desc = ("batch-wide compaction (fb_process_dev)" if args.config == 4 else
                       "batch-wide compaction (fb_parse_classify_dev)")
    traffic, traffic_tag = load_traffic(args.config, args.steps / main_r["launches"])
    if rank == 0:
        line = {
            "metric": "Mpackets/s device-resident header parse + 5-tuple classify, 64B & IMIX frames",
            "value": round(value, 2),
            "unit": "Mpackets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_r["elapsed"] * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic splitmix64 frames, SURVEY.md §8d)",
            "config": {"workload": WORKLOADS[args.config] + (" (Zipf(%g) flow popularity)" % args.zipf if args.zipf else ""), "frames_per_gpu_per_step": n,
                       "rotated_batches": rotate,
                       "batches_per_launch": round(args.steps / main_r["launches"], 2),
                       "batches_per_launch_max": bpl, "filter": "GlobalOnly",
                       "output": output_desc,
                       "parallelism": "packet-index shards x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_pmc_run": traffic_tag,
                         "algo_bytes_per_launch": int(algo_per_launch),
                         "kernel_ms_per_launch": round(per_launch_s * 1e3, 5),
                         "launches": main_r["launches"],
                         "timed_region_host_us_outside_kernels": main_r["host_us"],
                         "stream_copy_GBs": copy_gbs,
                         "frac_of_copy": round(achieved / copy_gbs, 4) if copy_gbs else None},
            "cpu_baseline": cpu,
            "batch_stats": main_r["stats"],
        }
        if world > 1:
            line["c5_ok"] = c5_ok
        if per_rank:
            line["per_rank"] = per_rank
            line["roofline"]["note"] = "rank 0's GPU; every rank's own fraction in per_rank"
        if extra:
            line["extra"] = extra
        _emit(line)
    if dist:
        dist.destroy_process_group()
    if not c5_ok:
        raise SystemExit("C5 exchange failed on some rank (c5_ok false in the line)")


if __name__ == "__main__":
    main()
