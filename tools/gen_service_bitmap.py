#!/usr/bin/env python3
"""Generate the 8 KiB service-port bitmap from the reference's embedded port table.

Run in the build container only (needs /root/reference, which does not exist on the
GPU box). The output `flodbadd_amd/data/service_ports.bin` is committed DATA: bit p is
set iff the reference's `get_name_from_port(p)` returns a non-empty name.

Reference semantics restated here:
  * src/port_vulns_db.rs:2-42179 -- `PORT_VULNS`, a JSON document embedded in a raw
    string; `vulnerabilities[]` entries carry `port` and `name`.
  * src/port_vulns.rs:51-76 -- `new_from_json` inserts EVERY entry into
    `PORT_NAMES_CACHE` (port -> name), including empty names; a later entry for the
    same port overwrites an earlier one (DashMap::insert).
  * src/port_vulns.rs:213-228 -- `get_name_from_port` returns the cached name, or ""
    for ports absent from the table.
  * src/packets.rs:233-237 -- "service port" <=> name is non-empty.

Layout: byte p >> 3, bit p & 7 (LSB first). Expected sha256:
04be3230d59a9c3dbe578f188b1f6113ebc188d8140f88fd6ea17dc595b32dad
"""
import hashlib
import json
import os
import sys

REF = "/root/reference/src/port_vulns_db.rs"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "flodbadd_amd", "data", "service_ports.bin")
# port -> non-empty name (what SessionInfo.dst_service holds, src/packets.rs:441-466)
NAMES_OUT = os.path.join(HERE, "..", "flodbadd_amd", "data", "service_names.json")
EXPECTED_SHA256 = "04be3230d59a9c3dbe578f188b1f6113ebc188d8140f88fd6ea17dc595b32dad"


def port_names(src_text: str) -> dict:
    start = src_text.index('r####"') + len('r####"')
    end = src_text.rindex('"####')
    doc = json.loads(src_text[start:end])
    names = {}
    for entry in doc["vulnerabilities"]:
        names[int(entry["port"])] = entry["name"]  # last insert wins
    return names


def build_bitmap(src_text: str) -> bytes:
    names = port_names(src_text)
    bm = bytearray(8192)
    for port, name in names.items():
        if name != "":
            bm[port >> 3] |= 1 << (port & 7)
    return bytes(bm)


def main() -> int:
    with open(REF, "r", encoding="utf-8") as f:
        text = f.read()
    bm = build_bitmap(text)
    digest = hashlib.sha256(bm).hexdigest()
    if digest != EXPECTED_SHA256:
        print(f"sha256 mismatch: {digest}", file=sys.stderr)
        return 1
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "wb") as f:
        f.write(bm)
    named = {str(p): n for p, n in sorted(port_names(text).items()) if n != ""}
    with open(NAMES_OUT, "w") as f:
        json.dump(named, f, separators=(",", ":"))
    print(f"wrote {NAMES_OUT} ({len(named)} names)")
    print(f"wrote {OUT} ({len(bm)} bytes, {sum(bin(b).count('1') for b in bm)} service ports, sha256 {digest})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
