"""CPU: the enrichment restatement (oracle/oracle.c orc_asn_* / orc_blacklist_mask) and the host
loaders (flodbadd_amd/enrich.py) against the reference's own known answers:
  src/asn.rs:82-200 (get_ipv4_asn 217.147.96.0 -> 174 COGENT-174, get_ipv6_asn 2001:200::1 ->
  2500 WIDE-BB, 0.0.0.0 -> None), and src/blacklists.rs:773-1240 (is_ip_blacklisted vectors,
  plain IPs as /32 and /128, local-range filtering at load).  The ASN rows are the ones the
  reference's test comments quote from its embedded IPtoASN tables (the tables themselves are
  not in the mount: .MISSING_LARGE_BLOBS)."""
import numpy as np

from flodbadd_amd import _native as N
from flodbadd_amd.enrich import asn_tables_from_tsv, blacklists_from_json, mask_names
from oracle import coracle

TSV = "\n".join([
    "0.0.0.0\t0.255.255.255\t0\tNone\tNot routed",
    "1.0.0.0\t1.0.0.255\t13335\tUS\tCLOUDFLARENET",
    "217.147.96.0\t217.147.111.255\t174\tUS\tCOGENT-174",
    "217.147.112.0\t217.147.127.255\t0\tNone\tNone",
    "2001:200::\t2001:200:5ff:ffff:ffff:ffff:ffff:ffff\t2500\tJP\tWIDE-BB WIDE Project",
    "2001:200:600::\t2001:200:6ff:ffff:ffff:ffff:ffff:ffff\t7667\tJP\tWIDE-BB",
    "short\trow",
    "9.9.9.9\t9.9.9.0\t1\tXX\tbad range (start > end)",
])


def _asn(ip, a4, a6, recs):
    r, _ = coracle.ip_lookup(a4, a6, np.zeros(0, dtype=N.CIDR_DTYPE), [ip])
    return None if r[0] < 0 else recs[int(r[0])]


def test_asn_known_answers():
    v4, v6, recs = asn_tables_from_tsv(TSV)
    assert len(v4) == 2 and len(v6) == 2  # Not routed / None owners, short and inverted rows skipped
    a4, a6 = coracle.asn_prepare(v4, 2), coracle.asn_prepare(v6, 10)
    assert _asn("217.147.96.0", a4, a6, recs) == (174, "US", "COGENT-174")
    assert _asn("2001:200::1", a4, a6, recs) == (2500, "JP", "WIDE-BB WIDE Project")
    assert _asn("0.0.0.0", a4, a6, recs) is None
    assert _asn("217.147.120.1", a4, a6, recs) is None


def test_asn_lookup_is_the_reference_binary_search():
    """Overlapping ranges: Db::lookup's probe sequence decides (not "any containing range")."""
    rows = ["10.0.0.0\t10.255.255.255\t1\tA\ta", "10.1.0.0\t10.1.0.255\t2\tB\tb", "10.2.0.0\t10.2.0.255\t3\tC\tc",
            "11.0.0.0\t11.0.0.255\t4\tD\td", "12.0.0.0\t12.0.0.255\t5\tE\te"]
    v4, _, recs = asn_tables_from_tsv("\n".join(rows))
    a4 = coracle.asn_prepare(v4, 2)
    # sorted: 10/8, 10.1/24, 10.2/24, 11/24, 12/24; mid = 2 (10.2.0.0/24) first
    got = {ip: _asn(ip, a4, a4[:0], recs) for ip in ("10.1.0.5", "10.3.0.1", "10.2.0.9", "10.0.0.1")}
    assert got["10.2.0.9"][0] == 3
    assert got["10.3.0.1"] is None  # 10/8 contains it, but the search walks right of mid and misses
    assert got["10.1.0.5"][0] in (1, 2)


def test_blacklist_known_answers():
    obj = {"blacklists": [
        {"name": "base_blacklist", "ip_ranges": ["192.168.0.0/16", "10.0.0.0/8", "8.8.8.8/32"]},
        {"name": "another_blacklist", "ip_ranges": ["172.16.0.0/12", "169.254.0.0/16", "9.9.9.9/32"]},
        {"name": "ipv6_blacklist", "ip_ranges": ["2001:db8::/32", "::1/128"]},
        {"name": "direct_ip_blacklist", "ip_ranges": ["192.168.1.1", "2001:db8::1", "10.0.0.0/8", "2001:db8:1::/64"]},
        {"name": "junk", "ip_ranges": ["not-a-range"]}]}
    cidrs, names = blacklists_from_json(obj, filter_local_ranges=False)
    ips = ["192.168.1.1", "1.2.3.4", "8.8.8.8", "172.16.1.1", "192.168.1.10", "2001:db8:1:2:3:4:5:6",
           "2002:db8:1:2:3:4:5:6", "::1", "2001:db8::1", "10.1.2.3", "2001:db8:1::abc", "192.168.1.2", "2001:db8::2"]
    none = np.zeros(0, dtype=N.ASN_RANGE_DTYPE)
    _, masks = coracle.ip_lookup(none, none, cidrs, ips)
    got = {ip: mask_names(m, names) for ip, m in zip(ips, masks)}
    assert got["192.168.1.1"] == ["base_blacklist", "direct_ip_blacklist"]
    assert got["1.2.3.4"] == []
    assert got["8.8.8.8"] == ["base_blacklist"]
    assert got["172.16.1.1"] == ["another_blacklist"]
    assert got["192.168.1.10"] == ["base_blacklist"]
    assert got["2001:db8:1:2:3:4:5:6"] == ["ipv6_blacklist"]
    assert got["2002:db8:1:2:3:4:5:6"] == []
    assert got["::1"] == ["ipv6_blacklist"]
    assert "direct_ip_blacklist" in got["2001:db8::1"] and "direct_ip_blacklist" in got["10.1.2.3"]
    assert "direct_ip_blacklist" in got["2001:db8:1::abc"]
    assert "direct_ip_blacklist" not in got["192.168.1.2"] and "direct_ip_blacklist" not in got["2001:db8::2"]


def test_blacklist_local_range_filter():
    """test_local_range_filtering (src/blacklists.rs:1072-1145): with filtering, ranges inside
    local space are dropped at load, public ones and plain public IPs kept."""
    obj = {"blacklists": [{"name": "filter_test_list", "ip_ranges": [
        "8.8.8.8/32", "203.0.113.45", "2001:db8::cafe", "192.168.0.0/16", "10.0.0.1", "172.16.0.0/12", "fc00::/7"]}]}
    cidrs, _ = blacklists_from_json(obj, filter_local_ranges=True)
    from flodbadd_amd.sessions import words_to_ip
    kept = {(str(words_to_ip(c["addr"], int(c["family"]))), int(c["prefix"])) for c in cidrs}
    assert kept == {("8.8.8.8", 32), ("203.0.113.45", 32), ("2001:db8::cafe", 128)}
