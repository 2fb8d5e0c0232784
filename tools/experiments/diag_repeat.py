"""Diagnostic: repeated device-resident launches of one batch must give identical stats/records."""
import sys, os, hashlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ctypes as C
from flodbadd_amd import _native as N, synth

cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 300
lib = N.gpu_lib()
cfg = N.FbConfig(); cfg.abi_version = 1; cfg.filter = 1; cfg.max_batch_packets = 1 << 24
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
frames, offs = synth.generate(cfgid, n)
s = N.Stream()
d_fr = N.DeviceBuffer(frames.nbytes).upload(frames); d_off = N.DeviceBuffer(offs.nbytes).upload(offs)
d_out = N.DeviceBuffer(n * 56); d_dns = N.DeviceBuffer(n * 16)
sts = [N.DeviceBuffer(128) for _ in range(iters)]
for i in range(iters):
    N.check(lib.fb_parse_classify_dev(ctx, d_fr.ptr, frames.nbytes, d_off.ptr, n, d_out.ptr, d_dns.ptr, None, sts[i].ptr, s.ptr))
s.sync()
ref = None
bad = 0
for i in range(iters):
    st = sts[i].download(np.zeros(1, dtype=N.STATS_DTYPE), stream=s.ptr)
    d = {k: int(st[0][k]) for k in N.STATS_FIELDS}
    if ref is None:
        ref = d; print("first", d)
    elif d != ref:
        bad += 1
        if bad < 10:
            print("launch", i, "diff", {k: (ref[k], d[k]) for k in d if d[k] != ref[k]})
print("bad launches:", bad, "of", iters)
