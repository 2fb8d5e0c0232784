"""Hand-built Ethernet frames for edge-case fixtures and the reference's known-answer tests."""
import ipaddress
import struct

import numpy as np

SYN, ACK, FIN, RST, PSH = 0x02, 0x10, 0x01, 0x04, 0x08
MACS = bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2])


def eth(ethertype, payload):
    return MACS + struct.pack("!H", ethertype) + payload


def ipv4(src, dst, proto, l4, ihl=5, total_length=None, options=b"", version=4):
    src, dst = ipaddress.IPv4Address(src), ipaddress.IPv4Address(dst)
    opts = options.ljust(max(ihl * 4 - 20, 0), b"\0")[: max(ihl * 4 - 20, 0)]
    tl = 20 + len(opts) + len(l4) if total_length is None else total_length
    hdr = struct.pack("!BBHHHBBH4s4s", (version << 4) | (ihl & 15), 0, tl & 0xFFFF, 0x1234, 0x4000, 64, proto, 0,
                      src.packed, dst.packed)
    return hdr + opts + l4


def ipv6(src, dst, nh, l4, payload_length=None):
    src, dst = ipaddress.IPv6Address(src), ipaddress.IPv6Address(dst)
    pl = len(l4) if payload_length is None else payload_length
    return struct.pack("!IHBB16s16s", 0x60000000, pl & 0xFFFF, nh, 64, src.packed, dst.packed) + l4


def tcp(sport, dport, flags, payload=b"", doff=5, options=b""):
    opts = options.ljust(max(doff * 4 - 20, 0), b"\0")[: max(doff * 4 - 20, 0)]
    return struct.pack("!HHIIBBHHH", sport, dport, 1, 2, (doff & 15) << 4, flags, 0xFFFF, 0, 0) + opts + payload


def udp(sport, dport, payload=b"", length=None):
    ln = 8 + len(payload) if length is None else length
    return struct.pack("!HHHH", sport, dport, ln & 0xFFFF, 0) + payload


def tcp_frame(src, sport, dst, dport, flags, payload_len, pad=0):
    """Realistic TCP frame (IHL 5 / doff 5) carrying `payload_len` payload bytes."""
    body = tcp(sport, dport, flags, bytes((i * 7) & 0xFF for i in range(payload_len)))
    ip = ipaddress.ip_address(src)
    if ip.version == 4:
        return eth(0x0800, ipv4(src, dst, 6, body)) + b"\0" * pad
    return eth(0x86DD, ipv6(src, dst, 6, body)) + b"\0" * pad


def udp_frame(src, sport, dst, dport, payload_len, pad=0):
    body = udp(sport, dport, bytes((i * 5) & 0xFF for i in range(payload_len)))
    ip = ipaddress.ip_address(src)
    if ip.version == 4:
        return eth(0x0800, ipv4(src, dst, 17, body)) + b"\0" * pad
    return eth(0x86DD, ipv6(src, dst, 17, body)) + b"\0" * pad


def pack(frames):
    """[bytes] -> (uint8 buffer, uint32 offsets[n+1])."""
    offs = np.zeros(len(frames) + 1, dtype=np.uint32)
    acc = 0
    for i, f in enumerate(frames):
        offs[i] = acc
        acc += len(f)
    offs[len(frames)] = acc
    buf = np.frombuffer(b"".join(frames), dtype=np.uint8).copy() if frames else np.zeros(0, np.uint8)
    return buf, offs


def edge_cases():
    """(name, frame bytes) covering every decode rule of SURVEY.md §8a a1 and the classifier."""
    A, B = "192.168.1.10", "8.8.8.8"
    V6A, V6B = "2001:db8::1", "2001:4860::8888"
    c = []
    c.append(("empty", b""))
    c.append(("short_13", bytes(13)))
    c.append(("eth_only_14", eth(0x0800, b"")))
    c.append(("arp", eth(0x0806, bytes(28))))
    c.append(("vlan_8100", eth(0x8100, struct.pack("!HH", 5, 0x0800) + ipv4(A, B, 6, tcp(1234, 80, ACK)))))
    c.append(("v4_ip_19B", eth(0x0800, bytes(19))))
    c.append(("v4_ip_20B_no_l4", eth(0x0800, ipv4(A, B, 6, b""))))
    c.append(("v4_tcp_19B", eth(0x0800, ipv4(A, B, 6, tcp(1234, 80, ACK)[:19]))))
    c.append(("v4_tcp_min", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, SYN)))))
    c.append(("v4_tcp_payload", tcp_frame(A, 40000, B, 443, PSH | ACK, 100)))
    c.append(("v4_tcp_eth_padding", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"xy"))) + bytes(20)))
    c.append(("v4_tot_lt_header", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"abcdef"), total_length=10))))
    c.append(("v4_tot_gt_caplen", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"abcdef"), total_length=1400))))
    c.append(("v4_ihl_0", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"hello"), ihl=0, total_length=45))))
    c.append(("v4_ihl_3", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"hello"), ihl=3, total_length=37))))
    c.append(("v4_ihl_6_options", eth(0x0800, ipv4(A, B, 6, tcp(40000, 443, ACK, b"opt"), ihl=6, options=b"\x01\x01\x01\x00"))))
    c.append(("v4_ihl_15_options", eth(0x0800, ipv4(A, B, 17, udp(5000, 6000, b"max"), ihl=15, options=b"\x01" * 40))))
    c.append(("v4_ihl_15_tcp", eth(0x0800, ipv4(A, B, 6, tcp(5001, 80, SYN | ACK, b"maxtcp"), ihl=15, options=b"\x01" * 40))))
    c.append(("v4_version_6_in_v4", eth(0x0800, ipv4(A, B, 6, tcp(1111, 2222, ACK), version=6))))
    c.append(("v4_icmp", eth(0x0800, ipv4(A, B, 1, bytes(8)))))
    c.append(("v4_udp_7B", eth(0x0800, ipv4(A, B, 17, udp(1, 2)[:7]))))
    c.append(("v4_udp_min", eth(0x0800, ipv4(A, B, 17, udp(5353, 5353)))))
    c.append(("v4_udp_len_field_ignored", eth(0x0800, ipv4(A, B, 17, udp(1000, 2000, b"abcdefgh", length=3)))))
    c.append(("v4_tcp_doff_15", eth(0x0800, ipv4(A, B, 6, tcp(3000, 80, ACK, b"d" * 50, doff=15)))))
    c.append(("v4_tcp_doff_gt_len", eth(0x0800, ipv4(A, B, 6, tcp(3000, 80, ACK, b"", doff=15)[:30]))))
    c.append(("v4_tcp_doff_2", eth(0x0800, ipv4(A, B, 6, tcp(3000, 80, ACK, b"abc", doff=2)))))
    c.append(("v4_dns_udp", udp_frame(A, 50000, B, 53, 30)))
    c.append(("v4_dns_udp_empty", udp_frame(A, 53, B, 50000, 0)))
    c.append(("v4_dns_tcp", tcp_frame(A, 50000, B, 53, PSH | ACK, 40)))
    c.append(("v4_dns_tcp_1B", tcp_frame(A, 50000, B, 53, PSH | ACK, 1)))
    c.append(("v4_dns_tcp_0B", tcp_frame(A, 53, B, 50000, ACK, 0)))
    c.append(("v4_dns_tcp_2B", tcp_frame(A, 53, B, 50000, ACK, 2)))
    c.append(("v6_ip_39B", eth(0x86DD, bytes(39))))
    c.append(("v6_tcp_min", eth(0x86DD, ipv6(V6A, V6B, 6, tcp(40000, 443, SYN)))))
    c.append(("v6_tcp_payload", tcp_frame(V6A, 40000, V6B, 443, PSH | ACK, 200)))
    c.append(("v6_udp", udp_frame(V6A, 40000, V6B, 123, 48)))
    c.append(("v6_plen_short", eth(0x86DD, ipv6(V6A, V6B, 17, udp(1, 2, b"abcdef"), payload_length=4))))
    c.append(("v6_plen_long", eth(0x86DD, ipv6(V6A, V6B, 17, udp(1, 2, b"abcdef"), payload_length=3000))))
    c.append(("v6_ext_hdr_hop", eth(0x86DD, ipv6(V6A, V6B, 0, bytes([6, 0]) + bytes(6) + tcp(1, 2, ACK)))))
    c.append(("v6_dns_tcp", tcp_frame(V6A, 53, V6B, 40000, ACK, 10)))
    c.append(("v6_linklocal_tcp", tcp_frame("fe80::1", 40000, "fe80::2", 22, ACK, 5)))
    c.append(("v6_ula_udp", udp_frame("fd12::1", 40000, "fd34::2", 5353, 5)))
    c.append(("v6_multicast", udp_frame("fe80::1", 5353, "ff02::fb", 5353, 20)))
    c.append(("v6_loopback", tcp_frame("::1", 40000, "::1", 8080, SYN, 0)))
    c.append(("v6_lan_prefix", tcp_frame("2001:db8:abcd:12::5", 40000, "2001:db8:abcd:12::1234", 22, ACK, 1)))
    c.append(("v6_lan_prefix_miss", tcp_frame("2001:db8:abcd:13::5", 40000, "2001:db8:abcd:12::1234", 22, ACK, 1)))
    # classifier cases
    c.append(("svc_src_swap", tcp_frame("1.1.1.1", 80, "192.168.1.1", 54321, ACK, 10)))
    c.append(("svc_both_syn_keep", tcp_frame("10.0.0.1", 80, "10.0.0.2", 443, SYN, 0)))
    c.append(("svc_both_synack_swap", tcp_frame("10.0.0.2", 443, "10.0.0.1", 80, SYN | ACK, 0)))
    c.append(("svc_both_ack_tiebreak_swap", tcp_frame("8.8.8.8", 80, "192.168.1.1", 12345, ACK, 200)))
    c.append(("svc_both_ack_tiebreak_keep", tcp_frame("192.168.1.1", 12345, "8.8.8.8", 80, ACK, 5)))
    c.append(("svc_both_udp_tiebreak", udp_frame("10.0.0.9", 123, "10.0.0.8", 5353, 12)))
    c.append(("svc_none_keep", tcp_frame("168.63.129.16", 44441, "10.1.0.40", 65535, SYN, 100)))
    c.append(("svc_empty_name_ports", tcp_frame("1.2.3.4", 54321, "5.6.7.8", 49152, ACK, 1)))
    c.append(("same_ip_same_port_swap", tcp_frame("10.0.0.5", 80, "10.0.0.5", 80, ACK, 3)))
    c.append(("same_ip_same_port_noswap", tcp_frame("10.0.0.5", 60001, "10.0.0.5", 60001, ACK, 3)))
    c.append(("tcp_flags_none", tcp_frame(A, 40001, B, 443, 0, 0)))
    c.append(("tcp_flags_rst", tcp_frame(A, 40001, B, 443, RST, 0)))
    c.append(("tcp_flags_fin_ack", tcp_frame(A, 40001, B, 443, FIN | ACK, 0)))
    c.append(("tcp_flags_all", tcp_frame(A, 40001, B, 443, 0xFF, 4)))
    c.append(("tcp_ack_only_resp", tcp_frame(B, 443, A, 40001, ACK, 0)))
    c.append(("lan_v4_172_16", tcp_frame("172.16.0.1", 40000, "172.31.255.255", 22, ACK, 1)))
    c.append(("lan_v4_172_32", tcp_frame("172.32.0.1", 40000, "172.15.0.1", 22, ACK, 1)))
    c.append(("lan_v4_linklocal_mcast", udp_frame("169.254.1.1", 5353, "224.0.0.251", 5353, 1)))
    c.append(("lan_v4_broadcast", udp_frame("0.0.0.0", 68, "255.255.255.255", 67, 300)))
    c.append(("lan_v4_240", udp_frame("240.0.0.1", 1000, "10.0.0.1", 2000, 1)))
    c.append(("loopback_v4", tcp_frame("127.0.0.1", 41000, "127.0.0.1", 8080, SYN, 10)))
    return c
