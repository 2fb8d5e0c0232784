"""Diagnostic (not product): KAT packets in several orders through the dense parsed path."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kat
from flodbadd_amd import _native as N
from flodbadd_amd.capture import FlodbaddGpuCapture, own_ip_table
from flodbadd_amd.sessions import SessionFilter, packets_to_parsed
from oracle import coracle

case = {c["name"]: c for c in kat.load()["cases"]}["test_session_management"]
lib = N.gpu_lib()
base = packets_to_parsed(kat.packets_of(case))
flt = SessionFilter.GlobalOnly
cap = FlodbaddGpuCapture(0, session_filter=flt, flow_capacity=0)
for order in ([0, 1, 2], [1, 0, 2], [1, 1, 1, 1], [0, 0, 1, 1], [2, 2, 2, 1], [1]):
    parsed = np.ascontiguousarray(base[order])
    n = len(parsed)
    d_in = N.DeviceBuffer(parsed.nbytes).upload(parsed)
    d_out = N.DeviceBuffer(64 * 56)
    d_cls = N.DeviceBuffer(64)
    d_st = N.DeviceBuffer(128)
    N.check(lib.fb_process_parsed_dev(cap.ctx, d_in.ptr, n, d_out.ptr, d_cls.ptr, d_st.ptr, None))
    dense_cls = d_cls.download(np.zeros(64, dtype=np.uint8))[:n].tolist()
    r_out, r_cls, r_st = coracle.process_parsed(coracle.make_cfg(int(flt)), parsed)
    print(order, "dense", dense_cls, "oracle", r_cls.tolist())
cap.close()
