#!/usr/bin/env python3
"""capture_sessions.py -- the counterpart of the reference's examples/capture_sessions.rs
(BASELINE.json configs[0]: capture over loopback, 10k synthetic 64-B TCP packets).

The reference example starts `FlodbaddCapture` on every interface, sleeps 5 s, calls `stop()`
and then `get_sessions(false)` (examples/capture_sessions.rs:33-50).  Two quirks make it print 0
sessions for loopback traffic: `FlodbaddCapture::new()` defaults the filter to GlobalOnly, which
drops loopback (src/capture.rs:108, src/packets.rs:323-324), and `stop()` clears the sessions
(src/capture.rs:383, 396).  This counterpart therefore uses SessionFilter.All and reads the sessions
before clearing them.

Capture: an AF_PACKET socket bound to `lo` (needs CAP_NET_RAW), outgoing copies skipped as
libpcap does on loopback, so each injected frame is seen once.  Traffic: `--packets` 64-B IPv4/TCP
frames injected on `lo` through a second AF_PACKET socket, `--flows` client ports against
127.0.0.1:8080 in both directions with SYN / SYN|ACK / ACK / PSH|ACK / FIN|ACK flags.  The captured
batch goes through the GPU path (`FlodbaddGpuCapture.process_frames`: parse + classify + session
table upsert); `--capture-only` skips the GPU (e.g. to write the batch with `--save`).
"""
import argparse
import os
import socket
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ETH_P_ALL = 0x0003
PACKET_OUTGOING = 4
MARK = b"FBADD"  # first payload bytes of every injected frame (their own traffic only is kept)
FLAGS = [0x02, 0x12, 0x10, 0x18, 0x11]  # SYN, SYN|ACK, ACK, PSH|ACK, FIN|ACK


def _csum(b):
    if len(b) & 1:
        b += b"\0"
    s = sum(struct.unpack("!%dH" % (len(b) // 2), b))
    s = (s >> 16) + (s & 0xFFFF)
    s += s >> 16
    return ~s & 0xFFFF


def frame(seq, n_flows):
    """The seq-th injected frame: 14 + 20 + 20 + 10 bytes = 64 B (IPv4 total_length 50)."""
    port = 40000 + seq % n_flows
    fl = FLAGS[(seq // n_flows) % len(FLAGS)]
    to_server = fl != 0x12 and (seq // n_flows) % 2 == 0 or fl == 0x02
    sport, dport = (port, 8080) if to_server else (8080, port)
    payload = MARK + struct.pack("!IB", seq, 0)
    lo = socket.inet_aton("127.0.0.1")
    tcp = struct.pack("!HHIIBBHHH", sport, dport, seq, 0, 5 << 4, fl, 65535, 0, 0) + payload
    ip = struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(tcp), seq & 0xFFFF, 0, 64, 6, 0, lo, lo)
    ip = ip[:10] + struct.pack("!H", _csum(ip)) + ip[12:]
    return b"\0" * 12 + b"\x08\x00" + ip + tcp


def capture_loopback(n_packets, n_flows, timeout=10.0):
    """Inject n_packets frames on lo and capture them back; returns (frames u8, offsets u32,
    seconds from the first send to the last frame captured)."""
    rx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
    tx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
    try:
        rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 64 << 20)
        rx.bind(("lo", 0))
        tx.bind(("lo", 0))
        rx.settimeout(0.05)
        buf, offs = bytearray(), [0]
        frames = [frame(k, n_flows) for k in range(n_packets)]
        t0 = time.perf_counter()
        got, sent, deadline = 0, 0, t0 + timeout
        while got < n_packets and time.perf_counter() < deadline:
            # inject in bursts the socket buffer holds (rmem_max caps SO_RCVBUF), then drain
            while sent < n_packets and sent - got < 128:
                tx.send(frames[sent])
                sent += 1
            try:
                data, addr = rx.recvfrom(65535)
            except socket.timeout:
                continue
            if addr[2] == PACKET_OUTGOING or len(data) < 59 or data[54:59] != MARK:
                continue  # libpcap skips outgoing copies on loopback; other traffic is not ours
            buf += data
            offs.append(len(buf))
            got += 1
        el = time.perf_counter() - t0
    finally:
        rx.close()
        tx.close()
    return np.frombuffer(bytes(buf), dtype=np.uint8).copy(), np.array(offs, dtype=np.uint32), el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=10000)
    ap.add_argument("--flows", type=int, default=100)
    ap.add_argument("--save", default=None, help="write the captured batch (frames, offsets) as .npz")
    ap.add_argument("--capture-only", action="store_true", help="no GPU: capture (and --save) only")
    a = ap.parse_args()
    try:
        frames, offs, el = capture_loopback(a.packets, a.flows)
    except PermissionError as e:
        raise SystemExit("AF_PACKET capture on lo needs CAP_NET_RAW: %s" % e)
    n = len(offs) - 1
    print("Captured %d of %d injected frames on lo in %.3f s (%.0f packets/s, host capture)" % (n, a.packets, el,
                                                                                               n / el))
    if a.save:
        np.savez_compressed(a.save, frames=frames, offsets=offs)
        print("wrote", a.save)
    if a.capture_only:
        return
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 16)
    try:
        t0 = time.perf_counter()
        r = cap.process_frames(frames, offs)
        t1 = time.perf_counter()
        sessions = cap.get_sessions()  # before clearing: the reference's stop() clears them
        print("GPU parse + classify + session upsert: %d frames, %d session records in %.3f ms (host-inclusive)"
              % (n, len(r.records), (t1 - t0) * 1e3))
        print("Captured %d session(s)." % len(sessions))
        cap.clear_all_sessions()
    finally:
        cap.close()


if __name__ == "__main__":
    main()
