"""Hand-built DNS messages (RFC 1035 wire format) for the DNS divert tests."""
import ipaddress
import struct


def name(n, ptr=None):
    """Labels of `n` ("" = root) + 0, or ending in a compression pointer to `ptr`."""
    out = b""
    for lab in [x for x in n.split(".") if x]:
        b = lab.encode("latin-1")
        out += bytes([len(b)]) + b
    return out + (struct.pack("!H", 0xC000 | ptr) if ptr is not None else b"\0")


def header(tx, qr, qd=0, an=0, ns=0, ar=0, flags=0x0100):
    return struct.pack("!HHHHHH", tx, flags | (0x8000 if qr else 0), qd, an, ns, ar)


def question(qname, qtype=1, qclass=1):
    return (qname if isinstance(qname, bytes) else name(qname)) + struct.pack("!HH", qtype, qclass)


def rr(rname, typ, rdata, cls=1, ttl=300):
    return (rname if isinstance(rname, bytes) else name(rname)) + struct.pack("!HHIH", typ, cls, ttl, len(rdata)) + rdata


def a(ip):
    return ipaddress.IPv4Address(ip).packed


def aaaa(ip):
    return ipaddress.IPv6Address(ip).packed


def opt(udp=1232, rdata=b""):
    return b"\0" + struct.pack("!HHBBHH", 41, udp, 0, 0, 0, len(rdata)) + rdata


def query(tx, qname, qtype=1, edns=True):
    return header(tx, False, qd=1, ar=1 if edns else 0) + question(qname, qtype) + (opt() if edns else b"")


def response(tx, qname, answers, qtype=1):
    """answers: list of ("A"|"AAAA"|"CNAME", value); owner names compress to the question (offset 12)."""
    body = b""
    for kind, v in answers:
        if kind == "A":
            body += rr(struct.pack("!H", 0xC00C), 1, a(v))
        elif kind == "AAAA":
            body += rr(struct.pack("!H", 0xC00C), 28, aaaa(v))
        else:
            body += rr(struct.pack("!H", 0xC00C), 5, name(v))
    return header(tx, True, qd=1, an=len(answers)) + question(qname, qtype) + body
