"""Independent pure-Python restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Written separately from oracle.c (different structure: `struct` slicing, the stdlib
`ipaddress` module for the LAN predicate, dict-based session table) so that agreement of the
two restatements is evidence about the rules, not about shared code.  Slow: small cases only.

Reference (edamametechnologies/flodbadd @ 2025-07-18):
  parse_packet_pcap         src/packets.rs:603-802 (pnet_packet 0.35.0 accessors; unpinned)
  process_parsed_packet     src/packets.rs:202-537
  update_session_stats      src/packets.rs:105-200
  map_tcp_flags / conn_state src/packets.rs:539-601
  is_lan_ip                 src/ip.rs:55-242
  get_name_from_port        src/port_vulns.rs:213-228
"""
import ipaddress
import struct

SYN, ACK, FIN, RST, PSH = 0x02, 0x10, 0x01, 0x04, 0x08

_V4_LAN = [ipaddress.ip_network(n) for n in (
    "0.0.0.0/32", "255.255.255.255/32", "127.0.0.0/8", "224.0.0.0/4", "169.254.0.0/16",
    "10.0.0.0/8", "172.16.0.0/12", "192.168.0.0/16")]
_V6_LAN = [ipaddress.ip_network(n) for n in ("::/128", "::1/128", "fe80::/10", "ff00::/8", "fc00::/7")]


class Config:
    def __init__(self, session_filter=2, service_ports=None, lan_v6=(), own_ips=()):
        self.filter = session_filter            # 0 LocalOnly, 1 GlobalOnly, 2 All
        self.service_ports = service_ports      # set of ports with a non-empty name
        self.lan_v6 = [ipaddress.IPv6Network("%s/%d" % (ip, p), strict=False) for ip, p in lan_v6]
        self.own_ips = {ipaddress.ip_address(x) for x in own_ips}

    @staticmethod
    def from_bitmap(bitmap, **kw):
        ports = {p for p in range(65536) if bitmap[p >> 3] & (1 << (p & 7))}
        return Config(service_ports=ports, **kw)

    def is_service(self, port):
        return port in self.service_ports

    def is_lan(self, ip):
        nets = _V4_LAN if ip.version == 4 else _V6_LAN + self.lan_v6
        return any(ip in n for n in nets)


def parse_packet_pcap(frame):
    """-> None | ("dns", payload_start, payload_len, proto, version)
            | ("session", proto, src, sport, dst, dport, packet_length, ip_packet_length, flags|None)"""
    if len(frame) < 14:
        return None
    (ethertype,) = struct.unpack_from("!H", frame, 12)
    ip = frame[14:]
    if ethertype == 0x0800:
        if len(ip) < 20:
            return None
        header_words = ip[0] & 0x0F
        (total_length,) = struct.unpack_from("!H", ip, 2)
        options = max(header_words * 4 - 20, 0)
        pay_len = max(total_length - header_words * 4, 0)
        begin = 20 + options
        payload = ip[begin:min(begin + pay_len, len(ip))] if len(ip) > begin else b""
        l4_start = 14 + begin
        src, dst = ipaddress.IPv4Address(ip[12:16]), ipaddress.IPv4Address(ip[16:20])
        proto, ip_len = ip[9], total_length
    elif ethertype == 0x86DD:
        if len(ip) < 40:
            return None
        (pl,) = struct.unpack_from("!H", ip, 4)
        payload = ip[40:min(40 + pl, len(ip))] if len(ip) > 40 else b""
        l4_start = 54
        src, dst = ipaddress.IPv6Address(ip[8:24]), ipaddress.IPv6Address(ip[24:40])
        proto, ip_len = ip[6], pl + 40
    else:
        return None
    if proto == 6:
        if len(payload) < 20:
            return None
        sport, dport = struct.unpack_from("!HH", payload, 0)
        data_offset = payload[12] >> 4
        hdr = data_offset * 4 if data_offset > 5 else 20
        body = payload[hdr:] if len(payload) > hdr else b""
        if 53 in (sport, dport):
            if len(body) < 2:
                return None
            return ("dns", l4_start + hdr + 2, len(body) - 2, 6, src.version)
        return ("session", 6, src, sport, dst, dport, len(body), ip_len, payload[13])
    if proto == 17:
        if len(payload) < 8:
            return None
        sport, dport = struct.unpack_from("!HH", payload, 0)
        if 53 in (sport, dport):
            return ("dns", l4_start + 8, len(payload) - 8, 17, src.version)
        return ("session", 17, src, sport, dst, dport, len(payload) - 8, ip_len, None)
    return None


def map_tcp_flags(flags, packet_length, orig):
    table = [(lambda f: f & SYN and not f & ACK, "S"), (lambda f: f & SYN and f & ACK, "H"),
             (lambda f: f & FIN, "F"), (lambda f: f & RST, "R")]
    for pred, ch in table:
        if pred(flags):
            return ch if orig else ch.lower()
    if packet_length > 0:
        return ">" if orig else "<"
    if flags & ACK:
        return "A" if orig else "a"
    return "-"


def conn_state(history):
    h = set(history)
    if {"S", "H", "F", "f"} <= h:
        return "SF"
    if "S" in h and "h" not in h and "r" not in h:
        return "S0"
    if "R" in h or "r" in h:
        return "REJ"
    if {"S", "H"} <= h and "F" not in h and "f" not in h:
        return "S1"
    return "-"


def canonical(cfg, proto, src, sport, dst, dport, flags):
    """Returns (key tuple, swapped) per src/packets.rs:232-311."""
    s_svc, d_svc = cfg.is_service(sport), cfg.is_service(dport)
    rev = (proto, dst, dport, src, sport)
    raw = (proto, src, sport, dst, dport)
    if s_svc and not d_svc:
        return rev, True
    if s_svc and d_svc:
        if flags is not None and proto == 6 and flags & SYN and not flags & ACK:
            return raw, False
        if flags is not None and proto == 6 and flags & SYN and flags & ACK:
            return rev, True
        return (rev, True) if sport < dport else (raw, False)
    return raw, False


def classify(cfg, parsed):
    """-> dict with key, swap, orig, meta bits, class ('session'|'filtered'), hist char."""
    _, proto, src, sport, dst, dport, plen, iplen, flags = parsed
    key, swap = canonical(cfg, proto, src, sport, dst, dport, flags)
    orig = (src, sport, dst, dport) == (key[1], key[2], key[3], key[4])
    local = cfg.is_lan(src) and cfg.is_lan(dst)
    if cfg.filter == 0 and not local:
        klass = "filtered"
    elif cfg.filter == 1 and local:
        klass = "filtered"
    else:
        klass = "session"
    return dict(key=key, swap=swap, orig=orig, klass=klass, plen=plen, iplen=iplen, flags=flags,
                local_src=cfg.is_lan(key[1]), local_dst=cfg.is_lan(key[3]),
                self_src=key[1] in cfg.own_ips, self_dst=key[3] in cfg.own_ips,
                dst_service=cfg.is_service(key[4]),
                hist=map_tcp_flags(flags, plen, orig) if flags is not None else None)


class SessionTable:
    """dict-based restatement of the DashMap upsert (src/packets.rs:329-535)."""

    def __init__(self):
        self.sessions = {}
        self.new = 0
        self.updated = 0

    def process(self, c, now=None):
        """now: the packet's capture time in ns (timed state: the 5-s segment timeout and the
        capture-time fields, src/packets.rs:137-200, 352-426), or None (positional model)."""
        key = c["key"]
        s = self.sessions.get(key)
        inserted = s is None
        if s is None:
            # is_local_src/dst and is_self_src/dst are stored once, at insert (src/packets.rs:429-435)
            s = dict(outbound_bytes=0, inbound_bytes=0, orig_pkts=0, resp_pkts=0, orig_ip_bytes=0,
                     resp_ip_bytes=0, history="", conn_state=None, segment_count=0, in_segment=True,
                     is_local_src=c["local_src"],
                     is_local_dst=c["local_dst"], is_self_src=c["self_src"], is_self_dst=c["self_dst"])
            self.sessions[key] = s
            self.new += 1
        else:
            self.updated += 1
        side = ("outbound_bytes", "orig_pkts", "orig_ip_bytes") if c["orig"] else \
               ("inbound_bytes", "resp_pkts", "resp_ip_bytes")
        s[side[0]] += c["plen"]
        s[side[1]] += 1
        s[side[2]] += c["iplen"]
        psh = c["flags"] is not None and c["key"][0] == 6 and bool(c["flags"] & PSH)
        if now is None:
            # segment end on TCP PSH (src/packets.rs:140-160 / 414-420; no wall-clock timeout here)
            s["segment_count"] += 1 if psh else 0
            s["in_segment"] = not psh
        elif inserted:  # src/packets.rs:352-380, 414-420
            s.update(start=now, last=now, end=None, seg_start=now, seg_end=None, ia_total=0.0, ia=0.0,
                     ia_ms=0, div=0, in_segment=not psh, segment_count=1 if psh else 0)
            if psh:
                s["seg_end"] = now
        else:  # update_session_stats, src/packets.rs:137-189
            def ms(a, b):  # chrono num_milliseconds: truncation toward zero
                d = a - b
                return d // 1000000 if d >= 0 else -((-d) // 1000000)
            timeout = ms(now, s["last"]) / 1000.0 >= 5.0
            is_end = psh or (s["in_segment"] and timeout)
            if not s["in_segment"]:
                s["in_segment"], s["seg_start"] = True, now
            if is_end and s["in_segment"]:
                prev = s["seg_end"]
                s["segment_count"] += 1
                s["in_segment"], s["seg_end"] = False, now
                if prev is not None:
                    ia_ms = ms(s["seg_start"], prev)
                    if ia_ms / 1000.0 >= 0.0:
                        s["ia_total"] += ia_ms / 1000.0
                        s["ia_ms"] += ia_ms
                        s["div"] = s["segment_count"] - 1 if s["segment_count"] > 1 else 0
                        s["ia"] = s["ia_total"] / (s["segment_count"] - 1) if s["segment_count"] > 1 else 0.0
                if timeout:
                    s["in_segment"], s["seg_start"] = True, now
            s["last"] = now
        if now is not None and c["flags"] is not None and c["flags"] & (FIN | RST) and s["end"] is None:
            s["end"] = now
        if c["flags"] is not None:
            s["history"] += c["hist"]
            if c["flags"] & (FIN | RST) and s["conn_state"] is None:
                s["conn_state"] = conn_state(s["history"])


def table_times(table):
    """Timed SessionTable -> {key: fb_flow_time fields}: start, last, end (None), segment start, last
    segment end (None), total interarrival (integer ms and the f64 running sum), divisor, segment
    count, in_segment."""
    return {k: (s["start"], s["last"], s["end"], s["seg_start"], s["seg_end"], s["ia_ms"], s["ia_total"], s["div"],
                s["segment_count"], s["in_segment"]) for k, s in table.sessions.items()}


def run_batch(cfg, frames, offsets, table=None, ts=None):
    """Whole-batch restatement: per frame class + emitted session records (dicts) + dns tuples."""
    classes, records, dns = [], [], []
    stats = dict(total_processed=0, tcp_processed=0, udp_processed=0, ipv4_processed=0, ipv6_processed=0,
                 n_session=0, n_dns=0, n_drop=0, n_filtered=0, bad_offsets=0)
    buf = bytes(frames)
    for i in range(len(offsets) - 1):
        a, b = int(offsets[i]), int(offsets[i + 1])
        if b < a or b > len(buf):
            classes.append(2)
            stats["n_drop"] += 1
            stats["bad_offsets"] += 1
            continue
        p = parse_packet_pcap(buf[a:b])
        if p is None:
            classes.append(2)
            stats["n_drop"] += 1
        elif p[0] == "dns":
            classes.append(1)
            stats["n_dns"] += 1
            dns.append((i, a + p[1], p[2], p[3], 2 if p[4] == 4 else 10))
        else:
            stats["total_processed"] += 1
            stats["tcp_processed" if p[1] == 6 else "udp_processed"] += 1
            stats["ipv4_processed" if p[2].version == 4 else "ipv6_processed"] += 1
            c = classify(cfg, p)
            c["pkt_index"] = i
            if c["klass"] == "filtered":
                classes.append(3)
                stats["n_filtered"] += 1
            else:
                classes.append(0)
                stats["n_session"] += 1
                records.append(c)
                if table is not None:
                    table.process(c, None if ts is None else int(ts[i]))
    return classes, records, dns, stats


def record_to_row(c, family_of=lambda ip: 2 if ip.version == 4 else 10):
    """Pack a classify() dict into the fb_pkt_out field values (for numpy comparison)."""
    def words(ip):
        if ip.version == 4:
            return [int(ip), 0, 0, 0]
        v = int(ip)
        return [(v >> (96 - 32 * k)) & 0xFFFFFFFF for k in range(4)]
    proto, src, sport, dst, dport = c["key"]
    meta = (1 if c["flags"] is not None else 0) | (2 if c["swap"] else 0) | (4 if c["orig"] else 0) | \
           (8 if c["local_src"] else 0) | (16 if c["local_dst"] else 0) | (32 if c["self_src"] else 0) | \
           (64 if c["self_dst"] else 0) | (128 if c["dst_service"] else 0)
    return dict(src_ip=words(src), dst_ip=words(dst), src_port=sport, dst_port=dport, protocol=proto,
                family=family_of(src), padding=0, packet_length=c["plen"], ip_packet_length=c["iplen"],
                tcp_flags=c["flags"] or 0, meta=meta, hist_char=ord(c["hist"]) if c["hist"] else 0,
                reserved=0, pkt_index=c["pkt_index"])


def table_rows(table):
    """SessionTable -> {canonical key tuple: counters + ordered state}, comparable with fb_flow_rec
    rows (see rows_of_flow_recs): the integer counters, history length, conn_state and the segment
    state."""
    out = {}
    for k, s in table.sessions.items():
        out[k] = (s["outbound_bytes"], s["inbound_bytes"], s["orig_pkts"], s["resp_pkts"], s["orig_ip_bytes"],
                  s["resp_ip_bytes"], len(s["history"]), s["conn_state"], s["segment_count"], s["in_segment"])
    return out


def rows_of_flow_recs(flows):
    """fb_flow_rec records (numpy, FLOW_REC_DTYPE) -> the same form as table_rows."""
    conn = {0: None, 1: "SF", 2: "S0", 3: "REJ", 4: "S1", 5: "-"}
    out = {}
    for r in flows:
        fam = int(r["family"])
        def ip(w):
            if fam == 2:
                return ipaddress.IPv4Address(int(w[0]))
            v = 0
            for x in w:
                v = (v << 32) | int(x)
            return ipaddress.IPv6Address(v)
        k = (int(r["protocol"]), ip(r["src_ip"]), int(r["src_port"]), ip(r["dst_ip"]), int(r["dst_port"]))
        out[k] = (int(r["outbound_bytes"]), int(r["inbound_bytes"]), int(r["orig_pkts"]), int(r["resp_pkts"]),
                  int(r["orig_ip_bytes"]), int(r["resp_ip_bytes"]), int(r["hist_len"]), conn[int(r["conn_state"])],
                  int(r["segment_count"]), bool(r["in_segment"]))
    return out

