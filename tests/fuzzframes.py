"""Mutated frames for parser fuzzing (test helper): valid synthetic frames of the C3 mix (IPv4 /
IPv6, TCP / UDP, DNS on port 53, 64 / 576 / 1500 B), each put through one of the mutations the
decode rules branch on: random bytes in the header window, truncation to a
random capture length, the EtherType set to IPv4 / IPv6 / something else, the IHL, total length,
IPv6 payload length and next header, the TCP data offset and flags, the ports (53 on either
side), both addresses made LAN / loopback / link-local / multicast (local sessions), and frames of
pure random bytes.  Deterministic for a seed."""
import random
import struct

import numpy as np

from flodbadd_amd import synth


def _mutate(f, rnd):
    f = bytearray(f)
    op = rnd.randrange(13)
    v6 = len(f) >= 14 and f[12:14] == b"\x86\xdd"
    l4 = 54 if v6 else 14 + 4 * (f[14] & 15 if len(f) > 14 else 5)
    if op == 0:  # random bytes in the header window
        for _ in range(rnd.randint(1, 6)):
            i = rnd.randrange(min(len(f), 96))
            f[i] = rnd.randrange(256)
    elif op == 1:  # truncation
        f = f[: rnd.randrange(len(f) + 1)]
    elif op == 2 and len(f) >= 14:  # EtherType
        f[12:14] = rnd.choice([b"\x08\x00", b"\x86\xdd", b"\x81\x00", b"\x08\x06", bytes([rnd.randrange(256)] * 2)])
    elif op == 3 and len(f) > 14 and not v6:  # IHL (0..15, so options and impossible values)
        f[14] = (f[14] & 0xF0) | rnd.randrange(16)
    elif op == 4 and len(f) >= 18 and not v6:  # IPv4 total length
        f[16:18] = struct.pack("!H", rnd.choice([0, 19, 20, 40, len(f) - 14, len(f), rnd.randrange(65536)]))
    elif op == 5 and len(f) >= 20 and v6:  # IPv6 payload length
        f[18:20] = struct.pack("!H", rnd.choice([0, 8, 20, len(f) - 54, rnd.randrange(65536)]))
    elif op == 6 and len(f) > 23:  # protocol / next header
        f[20 if v6 else 23] = rnd.choice([6, 17, 0, 1, 41, 43, 44, 58, 132, rnd.randrange(256)])
    elif op == 7 and len(f) > l4 + 13:  # TCP data offset (0..15) and flags
        f[l4 + 12] = (rnd.randrange(16) << 4) | (f[l4 + 12] & 15)
        f[l4 + 13] = rnd.randrange(256)
    elif op == 8 and len(f) > l4 + 3:  # a port to / from 53 (DNS divert) or a service / ephemeral port
        p = rnd.choice([53, 53, 80, 443, 0, 65535, rnd.randrange(65536)])
        j = l4 + rnd.choice([0, 2])
        f[j: j + 2] = struct.pack("!H", p)
    elif op == 9:  # pure random bytes
        f = bytearray(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 13, 14, 33, 34, 54, 60, 64, 90])))
    elif op == 10 and len(f) > l4 + 3:  # DNS over a short payload: port 53 and a truncation right after L4
        f[l4: l4 + 2] = struct.pack("!H", 53)
        f = f[: rnd.randrange(l4, min(len(f), l4 + 24) + 1)]
    elif op == 11 and len(f) >= (54 if v6 else 34):  # both addresses LAN (or loopback / link-local / multicast)
        if v6:
            for j in (22, 38):
                f[j: j + 16] = rnd.choice([bytes.fromhex("fe80") + bytes(rnd.randrange(256) for _ in range(14)),
                                           bytes(15) + b"\x01", bytes.fromhex("fd12") + bytes(14),
                                           bytes.fromhex("ff02") + bytes(13) + b"\x01"])
        else:
            for j in (26, 30):
                f[j: j + 4] = rnd.choice([bytes([10, rnd.randrange(256), 0, 1]), bytes([192, 168, 1, rnd.randrange(256)]),
                                          bytes([127, 0, 0, 1]), bytes([172, 16 + rnd.randrange(16), 0, 9]),
                                          bytes([169, 254, 3, 4]), bytes([224, 0, 0, 251]), bytes(4), bytes([255] * 4)])
    # op 12 (and inapplicable ops): the frame unchanged
    return bytes(f)


def generate(n, seed):
    """n mutated frames -> (frames u8, offsets u32[n+1])."""
    rnd = random.Random(seed)
    frames, offs = synth.generate(3, n, first=seed * n)
    out, o = [], [0]
    for i in range(n):
        g = _mutate(frames[offs[i]: offs[i + 1]].tobytes(), rnd)
        out.append(g)
        o.append(o[-1] + len(g))
    buf = np.frombuffer(b"".join(out), dtype=np.uint8).copy() if o[-1] else np.zeros(0, dtype=np.uint8)
    return buf, np.array(o, dtype=np.uint32)
