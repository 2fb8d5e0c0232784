"""CPU: the all-cores baseline (orc_parse_classify_mt) returns exactly the
single-thread oracle's outputs (records and DNS side records in packet order, batch stats)."""
import ctypes as C

import numpy as np
import pytest

from flodbadd_amd import synth
from oracle import coracle


@pytest.mark.parametrize("cid,threads", [(2, 4), (3, 7), (3, 1)])
def test_mt_equals_single(cid, threads):
    frames, offs = synth.generate(cid, 30011)
    cfg = coracle.make_cfg(1)
    r_out, r_dns, _, r_st = coracle.parse_classify(cfg, frames, offs)
    n = len(offs) - 1
    out = np.zeros(n, dtype=coracle.PKT_OUT_DTYPE)
    dns = np.zeros(n, dtype=coracle.DNS_OUT_DTYPE)
    st = np.zeros(1, dtype=coracle.STATS_DTYPE)
    no, nd = C.c_uint32(), C.c_uint32()
    coracle.lib().orc_parse_classify_mt(C.byref(cfg), frames.ctypes.data, frames.nbytes, offs.ctypes.data, n,
                                        out.ctypes.data, C.byref(no), dns.ctypes.data, C.byref(nd),
                                        st.ctypes.data, threads)
    assert out[: no.value].tobytes() == r_out.tobytes()
    assert dns[: nd.value].tobytes() == r_dns.tobytes()
    assert st.tobytes() == r_st.tobytes()


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_pipeline_mt_tables_union_equals_single(threads):
    """orc_pipeline_mt (the all-cores C4 baseline: parse + classify + session upsert, each thread
    owning a share of the keys) builds exactly the single-thread table, split across threads."""
    frames, offs = synth.generate(4, 40000)
    cfg = coracle.make_cfg(1)
    r_out, _, _, r_st = coracle.parse_classify(cfg, frames, offs)
    ref = coracle.Flows()
    st1 = np.zeros(1, dtype=coracle.STATS_DTYPE)
    ref.update(r_out, st1)
    tables, st = coracle.pipeline_mt(cfg, frames, offs, threads)
    rows = np.concatenate([t.export_sorted() for t in tables])
    key = lambda a: sorted(a[i].tobytes() for i in range(len(a)))
    assert key(rows) == key(ref.export_sorted())
    assert int(st[0]["new_sessions"]) == int(st1[0]["new_sessions"])
    assert int(st[0]["updated_sessions"]) == int(st1[0]["updated_sessions"])
    assert int(st[0]["n_session"]) == int(r_st[0]["n_session"])
