"""CPU-side checks of the C-ABI boundary: the library loads (no GPU needed for dlopen) and exports
exactly the functions include/flodbadd_gpu.h declares; record layouts match the header."""
import ctypes as C
import os
import re
import subprocess

import numpy as np

from flodbadd_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "flodbadd_gpu.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(fb_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_all_bound_symbols():
    declared = _declared_functions()
    bound = sorted(n for n, _, _ in N.GPU_SYMBOLS)
    assert declared == bound, (set(declared) ^ set(bound))


def test_integration_rust_binding_declares_every_entry_point():
    """INTEGRATION.md's Rust extern blocks bind every function of the header (a maintainer copying
    them gets the whole ABI)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    rust = "\n".join(re.findall(r"```rust\n(.*?)```", doc, flags=re.S))
    declared_rust = set(re.findall(r"pub fn (fb_\w+)\s*\(", rust))
    missing = set(_declared_functions()) - declared_rust
    assert not missing, sorted(missing)


def test_library_exports_every_declared_symbol():
    from flodbadd_amd.build import build_gpu
    build_gpu()
    lib = N.gpu_lib()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.GPU_LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (fb_\w+)", out))
    assert set(_declared_functions()) <= exported
    assert lib.fb_abi_version() == N.FB_ABI_VERSION


def test_no_gpu_means_loud_failure():
    """Without a gfx950 device fb_create must fail (no CPU fallback anywhere)."""
    lib = N.gpu_lib()
    n = C.c_int(-1)
    assert lib.fb_device_count(C.byref(n)) == 0
    if n.value == 0:
        cfg = N.FbConfig()
        cfg.abi_version = N.FB_ABI_VERSION
        cfg.filter = N.FB_FILTER_ALL
        assert not lib.fb_create(0, C.byref(cfg))
        assert lib.fb_last_error()


def test_invalid_arguments_are_errors_not_aborts():
    lib = N.gpu_lib()
    assert lib.fb_set_filter(None, 0) == N.FB_ERR_INVAL
    assert lib.fb_destroy(None) == N.FB_ERR_INVAL
    assert lib.fb_parse_classify_dev(None, None, 0, None, 0, None, None, None, None, None) == N.FB_ERR_INVAL
    cfg = N.FbConfig()
    cfg.abi_version = 999
    assert not lib.fb_create(0, C.byref(cfg))
    assert b"abi_version" in lib.fb_last_error()


def test_record_layouts():
    assert N.PKT_OUT_DTYPE.itemsize == 56
    assert N.PKT_OUT_DTYPE.fields["packet_length"][1] == 40
    assert N.PKT_OUT_DTYPE.fields["pkt_index"][1] == 52
    assert N.FLOW_REC_DTYPE.fields["outbound_bytes"][1] == 40
    assert N.FLOW_REC_DTYPE.itemsize == 136
    for f, off in (("first_seen", 88), ("last_seen", 96), ("end_seen", 104), ("hist_len", 112),
                   ("hist_mask", 116), ("conn_state", 118), ("slot", 120), ("segment_count", 128),
                   ("in_segment", 132)):
        assert N.FLOW_REC_DTYPE.fields[f][1] == off, f
    assert N.DNS_OUT_DTYPE.itemsize == 16
    assert N.STATS_DTYPE.itemsize == 128


def test_record_layouts_match_the_header(tmp_path):
    """The numpy dtypes the host side uses are the C header's structs: offsetof / sizeof of
    include/flodbadd_gpu.h compiled by gcc here."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    checks = [("fb_flow_rec", N.FLOW_REC_DTYPE), ("fb_flow_mrec", N.FLOW_MREC_DTYPE), ("fb_pkt_out", N.PKT_OUT_DTYPE),
              ("fb_batch_stats", N.STATS_DTYPE), ("fb_dns_out", N.DNS_OUT_DTYPE)]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s/include/flodbadd_gpu.h"' % root, "int main(void) {"]
    want = []
    for st, dt in checks:
        src.append('printf("%%zu\\n", sizeof(%s));' % st)
        want.append(dt.itemsize)
        for f in dt.names:
            if f in ("src_ip", "dst_ip", "src_port", "dst_port", "protocol", "family", "padding") or f.startswith("reserved"):
                continue  # the key's fields (fb_session_key: its size below) and reserved words
            src.append('printf("%%zu\\n", offsetof(%s, %s));' % (st, f))
            want.append(dt.fields[f][1])
    src.append('printf("%zu\\n", sizeof(fb_session_key)); return 0; }')
    want.append(40)
    c = tmp_path / "lay.c"
    c.write_text("\n".join(src) + "\n")
    subprocess.run(["gcc", "-o", str(tmp_path / "lay"), str(c)], check=True)
    got = [int(x) for x in subprocess.run([str(tmp_path / "lay")], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert got == want


def test_flow_hash_is_deterministic_and_host_side():
    lib = N.gpu_lib()
    k = np.zeros(1, dtype=N.PKT_OUT_DTYPE)
    k[0]["src_ip"][0] = 0xC0A80101
    k[0]["dst_ip"][0] = 0x08080808
    k[0]["src_port"], k[0]["dst_port"], k[0]["protocol"], k[0]["family"] = 12345, 80, 6, 2
    h1 = lib.fb_flow_hash(N.ptr(k))
    h2 = lib.fb_flow_hash(N.ptr(k.copy()))
    assert h1 == h2 and h1 != 0
    k[0]["dst_port"] = 81
    assert lib.fb_flow_hash(N.ptr(k)) != h1


def test_header_constants_match_python():
    import re
    hdr = open(os.path.join(ROOT, "include", "flodbadd_gpu.h")).read()
    for name in ("FB_MAX_SEG_BATCHES", "FB_SEG_FRAMES", "FB_ABI_VERSION"):
        m = re.search(r"#define %s (\d+)u" % name, hdr)
        assert m and int(m.group(1)) == getattr(N, name), name


def test_bench_launch_plan():
    """bench.plan_launches: k steps in ceil(k / bpl) launches of near-equal size."""
    import bench
    for bpl in (1, 8, 12, 32):
        for k in list(range(0, 70)) + [200, 1000]:
            p = bench.plan_launches(k, bpl)
            assert sum(p) == k and all(1 <= c <= bpl for c in p)
            assert len(p) == -(-k // bpl) and (not p or max(p) - min(p) <= 1)


def test_bandwidth_reference_is_outside_the_product():
    """bench.py's stream-copy reference lives in its own library (libfb_bwref.so), not in the C ABI."""
    from flodbadd_amd.build import build_bwref
    path = build_bwref()
    lib = C.CDLL(path)
    assert hasattr(lib, "fb_bwref_copy")
    out = subprocess.run(["nm", "-D", "--defined-only", N.GPU_LIB_PATH], capture_output=True, text=True).stdout
    assert "fb_bwref" not in out
    lib.fb_bwref_copy.restype = C.c_int
    lib.fb_bwref_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    assert lib.fb_bwref_copy(None, None, 16, 1, None) != 0  # invalid arguments: an error, no launch
