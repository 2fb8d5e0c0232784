"""DNS divert on the GPU + the reference's bookkeeping on the host.

`parse_dns` runs fb_dns_parse_dev over a batch's DNS side records (the port-53 payloads that
parse_packet_pcap diverts, src/packets.rs:638-650, 681-686); `DnsResolver.process` then applies,
in packet order, what DnsPacketProcessor::process_dns_packet does with each parsed packet
(src/dns.rs:35-99): a query's first question name is remembered under the transaction id
(reverse lookups excluded), a response takes that name back and maps each A / AAAA answer to it.
Packets DnsPacket::parse rejects are skipped (the reference logs a warning).  The expiry of
pending queries (30 s, src/dns.rs:101-121) is wall-clock bookkeeping left to the caller
(`expire`).
"""
import numpy as np

from . import _native as N
from .sessions import words_to_ip


def parse_dns(frames, dns_records):
    """GPU parse of DNS_OUT_DTYPE records over their frame buffer -> (msgs, names, addrs)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    dns_records = np.ascontiguousarray(dns_records, dtype=N.DNS_OUT_DTYPE)
    n = len(dns_records)
    if n == 0:
        return np.zeros(0, dtype=N.DNS_MSG_DTYPE), np.zeros((0, N.FB_DNS_MAX_NAME), np.uint8), \
            np.zeros((0, N.FB_DNS_MAX_ADDRS), dtype=N.FB_IP_DTYPE)
    lib = N.gpu_lib()
    d_fr = N.DeviceBuffer(max(frames.nbytes, 1))
    if frames.nbytes:
        d_fr.upload(frames)
    d_dns = N.DeviceBuffer(dns_records.nbytes).upload(dns_records)
    d_msg = N.DeviceBuffer(n * N.DNS_MSG_DTYPE.itemsize)
    d_names = N.DeviceBuffer(n * N.FB_DNS_MAX_NAME)
    d_addrs = N.DeviceBuffer(n * N.FB_DNS_MAX_ADDRS * N.FB_IP_DTYPE.itemsize)
    N.check(lib.fb_dns_parse_dev(_ctx(), d_fr.ptr, frames.nbytes, d_dns.ptr, n, None, d_msg.ptr, d_names.ptr,
                                 d_addrs.ptr, None))
    msgs = d_msg.download(np.zeros(n, dtype=N.DNS_MSG_DTYPE))
    names = d_names.download(np.zeros((n, N.FB_DNS_MAX_NAME), dtype=np.uint8))
    addrs = d_addrs.download(np.zeros((n, N.FB_DNS_MAX_ADDRS), dtype=N.FB_IP_DTYPE))
    return msgs, names, addrs


_CTX = None


def _ctx():
    """A small context for parse_dns (no flow table)."""
    global _CTX
    if _CTX is None:
        from .capture import FlodbaddGpuCapture
        _CTX = FlodbaddGpuCapture(0, flow_capacity=0)
    return _CTX.ctx


class DnsResolver:
    """The bookkeeping of DnsPacketProcessor (src/dns.rs:16-99) over parsed messages."""

    def __init__(self):
        self.pending = {}      # transaction id -> domain name (pending_dns_queries)
        self.resolutions = {}  # ip -> domain name (dns_resolutions)

    def process(self, msgs, names, addrs):
        for i, m in enumerate(msgs):
            if int(m["status"]) != 0:
                continue  # "Failed to parse DNS packet"
            tx = int(m["id"])
            if int(m["flags"]) & N.DNS_QUERY:
                if int(m["flags"]) & N.DNS_HAS_QUESTION and not int(m["flags"]) & N.DNS_REVERSE:
                    self.pending[tx] = bytes(names[i][: int(m["name_len"])]).decode("ascii")
            else:
                name = self.pending.pop(tx, None)
                if name is None:
                    continue
                for a in addrs[i][: int(m["n_addrs"])]:
                    self.resolutions[words_to_ip(a["addr"], int(a["family"]))] = name

    def expire(self, ids):
        """Drop pending queries (the reference's 30-s cleanup task)."""
        for t in ids:
            self.pending.pop(t, None)
