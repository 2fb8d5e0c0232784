"""Deterministic synthetic capture batches via libfb_synth.so.

Configs (BASELINE.json `configs`):
  C2: 1M x 64-B IPv4/TCP, flow pool 2^16             -> config_id 2, mode 0
  C3: 1M IMIX 64/576/1500 (7:4:1), v4/v6, TCP/UDP     -> config_id 3, mode 1
  C4: 10M IMIX + flow table, pool 2^20 (uniform/Zipf) -> config_id 4, mode 1
  C5: 80M = 8 x 10M shards by packet index            -> config_id 5, mode 1
Override lan_dst_permille (e.g. 800) for a LAN-heavy variant in which the Local/Global filters
drop a large share of the batch.
"""
import ctypes as C
import os

import numpy as np

from ._native import SYNTH_LIB_PATH, NativeLibraryMissing


class SynthCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_flows", C.c_uint32), ("mode", C.c_uint32),
                ("v6_permille", C.c_uint32), ("udp_permille", C.c_uint32), ("dns_permille", C.c_uint32),
                ("zipf", C.c_uint32), ("zipf_s", C.c_double), ("lan_dst_permille", C.c_uint32)]


CONFIGS = {
    2: dict(n_flows=1 << 16, mode=0, v6_permille=0, udp_permille=0, dns_permille=5, zipf=0, zipf_s=1.1),
    3: dict(n_flows=1 << 16, mode=1, v6_permille=200, udp_permille=300, dns_permille=5, zipf=0, zipf_s=1.1),
    4: dict(n_flows=1 << 20, mode=1, v6_permille=200, udp_permille=300, dns_permille=5, zipf=0, zipf_s=1.1),
    5: dict(n_flows=1 << 20, mode=1, v6_permille=200, udp_permille=300, dns_permille=5, zipf=0, zipf_s=1.1),
}

_lib = None


def _synth():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_LIB_PATH):
            raise NativeLibraryMissing("%s missing: run `python -m flodbadd_amd.build`" % SYNTH_LIB_PATH)
        lib = C.CDLL(SYNTH_LIB_PATH)
        lib.fb_synth_plan.restype = C.c_uint64
        lib.fb_synth_plan.argtypes = [C.POINTER(SynthCfg), C.c_uint64, C.c_uint32, C.c_void_p]
        lib.fb_synth_fill.restype = C.c_int
        lib.fb_synth_fill.argtypes = [C.POINTER(SynthCfg), C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int]
        lib.fb_synth_flow_of.restype = C.c_uint32
        lib.fb_synth_flow_of.argtypes = [C.POINTER(SynthCfg), C.c_uint64]
        _lib = lib
    return _lib


def make_cfg(config_id, **overrides):
    d = dict(CONFIGS[config_id])
    d.update(overrides)
    return SynthCfg(seed=0xF10DBADD ^ config_id, **d)


def generate(config_id, n, first=0, threads=None, frames_out=None, **overrides):
    """Return (frames uint8[bytes], offsets uint32[n+1]) for packets [first, first+n).

    `frames_out`, if given, is a preallocated uint8 buffer (e.g. pinned) of sufficient size."""
    cfg = make_cfg(config_id, **overrides)
    lib = _synth()
    offsets = np.empty(n + 1, dtype=np.uint32)
    total = lib.fb_synth_plan(C.byref(cfg), first, n, offsets.ctypes.data)
    if total >= 1 << 32:
        raise ValueError("batch exceeds 4 GiB (u32 offsets)")
    if frames_out is None:
        frames = np.empty(max(total, 1), dtype=np.uint8)[:total]
    else:
        if frames_out.nbytes < total:
            raise ValueError("frames_out holds %d bytes, the batch needs %d" % (frames_out.nbytes, total))
        frames = frames_out[:total]
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    lib.fb_synth_fill(C.byref(cfg), first, n, offsets.ctypes.data, frames.ctypes.data, threads)
    return frames, offsets


def dns_workload(n, seed=0xD115):
    """A device-benchmark DNS divert batch: `n` port-53 payloads (RFC 1035 wire format) and their
    DNS_OUT_DTYPE side records, cycling through 512 distinct messages: queries (A / AAAA / PTR,
    with and without EDNS) and responses (CNAME chain + A / AAAA answers, compression pointers),
    the shapes src/dns.rs handles.  Returns (payload uint8[bytes], records)."""
    import struct
    from . import _native as N
    rnd = np.random.default_rng(seed)

    def name(s, ptr=None):
        out = b"".join(bytes([len(x)]) + x.encode() for x in s.split(".") if x)
        return out + (struct.pack("!H", 0xC000 | ptr) if ptr is not None else b"\0")

    def rr(owner, typ, rdata):
        return owner + struct.pack("!HHIH", typ, 1, 300, len(rdata)) + rdata

    msgs = []
    for i in range(512):
        tx = int(rnd.integers(0, 1 << 16))
        host = "h%d.svc%d.example%d.com" % (i, i % 37, i % 5)
        kind = i % 4
        if kind == 0:    # A query with EDNS
            m = struct.pack("!HHHHHH", tx, 0x0100, 1, 0, 0, 1) + name(host) + struct.pack("!HH", 1, 1) + \
                b"\0" + struct.pack("!HHBBHH", 41, 1232, 0, 0, 0, 0)
        elif kind == 1:  # AAAA query
            m = struct.pack("!HHHHHH", tx, 0x0100, 1, 0, 0, 0) + name(host) + struct.pack("!HH", 28, 1)
        elif kind == 2:  # reverse lookup
            m = struct.pack("!HHHHHH", tx, 0x0100, 1, 0, 0, 0) + \
                name("%d.%d.0.10.in-addr.arpa" % (i & 255, i >> 8)) + struct.pack("!HH", 12, 1)
        else:            # response: CNAME + 2 A + 1 AAAA, names compressed against the question
            q = name(host) + struct.pack("!HH", 1, 1)
            an = rr(b"\xc0\x0c", 5, name("edge%d.cdn.example.net" % i)) + \
                rr(b"\xc0\x0c", 1, struct.pack("!I", 0x5DB8D800 | (i & 255))) + \
                rr(b"\xc0\x0c", 1, struct.pack("!I", 0x5DB8D900 | (i & 255))) + \
                rr(b"\xc0\x0c", 28, bytes([0x26, 0x06, 0x28, 0]) + bytes(11) + bytes([i & 255]))
            m = struct.pack("!HHHHHH", tx, 0x8180, 1, 4, 0, 0) + q + an
        msgs.append(m)
    lens = np.array([len(m) for m in msgs], dtype=np.uint64)
    base = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    reps = (n + 511) // 512
    payload = np.tile(base, reps)
    idx = np.arange(n, dtype=np.uint64)
    rec = np.zeros(n, dtype=N.DNS_OUT_DTYPE)
    rec["pkt_index"] = idx
    rec["payload_offset"] = (idx // 512) * np.uint64(base.nbytes) + starts[idx % 512]
    rec["payload_length"] = lens[idx % 512]
    rec["protocol"] = 17
    rec["family"] = 2
    return payload, rec
