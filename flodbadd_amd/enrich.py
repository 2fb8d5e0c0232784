"""Host side of the new-session enrichment: the reference's table loaders
restated for the C ABI's fb_asn_range / fb_cidr tables, and the capture-level calls.

  asn_tables_from_tsv   Db::from_tsv (src/asn_db.rs:82-140): IPtoASN TSV rows
                        `range_start range_end as_number country owner`; rows with < 5 fields or
                        owner "Not routed" / "None" skipped, mismatched families or start > end
                        skipped (the sort happens in fb_set_asn_tables, stable like Vec::sort).
  blacklists_from_json  Blacklists::new_from_json (src/blacklists.rs:111-186): a plain IP becomes
                        /32 or /128, unparsable ranges are skipped, and with filter_local_ranges
                        a range entirely inside a known local range is dropped
                        (is_range_local_to_filter, src/blacklists.rs:70-105).
"""
import ipaddress

import numpy as np

from . import _native as N
from .sessions import ip_to_words

LOCAL_V4_TO_FILTER = [ipaddress.ip_network(x) for x in ("0.0.0.0/8", "10.0.0.0/8", "127.0.0.0/8", "169.254.0.0/16",
                                                        "172.16.0.0/12", "192.168.0.0/16")]
LOCAL_V6_TO_FILTER = [ipaddress.ip_network(x) for x in ("::/128", "::1/128", "fc00::/7", "fe80::/10")]


def asn_tables_from_tsv(text):
    """-> (v4 ASN_RANGE_DTYPE array, v6 array, records [(as_number, country, owner)]), file order."""
    v4, v6, recs = [], [], []
    for line in text.splitlines():
        f = line.split("\t")
        if len(f) < 5:
            continue
        owner = f[4]
        if owner in ("Not routed", "None"):
            continue
        a, b = ipaddress.ip_address(f[0]), ipaddress.ip_address(f[1])  # parse errors abort, like `?`
        asn = int(f[2])
        if a.version != b.version or a > b:
            continue
        r = np.zeros(1, dtype=N.ASN_RANGE_DTYPE)[0]
        r["start"] = ip_to_words(a)[0]
        r["end"] = ip_to_words(b)[0]
        r["as_number"] = asn
        r["record"] = len(recs)
        recs.append((asn, f[3], owner))
        (v4 if a.version == 4 else v6).append(r)
    mk = lambda rows: np.array(rows, dtype=N.ASN_RANGE_DTYPE) if rows else np.zeros(0, dtype=N.ASN_RANGE_DTYPE)
    return mk(v4), mk(v6), recs


def _is_range_local(net):
    return any(net.version == l.version and net.subnet_of(l)
               for l in (LOCAL_V4_TO_FILTER if net.version == 4 else LOCAL_V6_TO_FILTER))


def blacklists_from_json(obj, filter_local_ranges=False):
    """{"blacklists": [{"name": ..., "ip_ranges": [...]}, ...]} -> (CIDR_DTYPE array, [names])."""
    names, rows = [], []
    for info in obj["blacklists"]:
        if len(names) >= N.FB_MAX_BLACKLISTS:
            raise ValueError("at most %d blacklists" % N.FB_MAX_BLACKLISTS)
        lid = len(names)
        names.append(info["name"])
        for s in info.get("ip_ranges", []):
            try:
                ip = ipaddress.ip_address(s)
                s = "%s/%d" % (s, 32 if ip.version == 4 else 128)
            except ValueError:
                pass
            try:
                net = ipaddress.ip_network(s, strict=False)
                addr = ipaddress.ip_address(s.split("/")[0])
            except ValueError:
                continue  # "Failed to parse IP range" (src/blacklists.rs:151-157)
            if filter_local_ranges and _is_range_local(net):
                continue
            r = np.zeros(1, dtype=N.CIDR_DTYPE)[0]
            r["addr"], r["family"] = ip_to_words(addr)
            r["prefix"] = net.prefixlen
            r["list"] = lid
            rows.append(r)
    arr = np.array(rows, dtype=N.CIDR_DTYPE) if rows else np.zeros(0, dtype=N.CIDR_DTYPE)
    return arr, names


def mask_names(mask, names):
    """The list names of a blacklist bit mask (is_ip_blacklisted's Vec<String>)."""
    return [n for i, n in enumerate(names) if (int(mask) >> i) & 1]
