#!/bin/bash
# round 6: the timed / routed / ring tests, then the ring bench leg alone
mkdir -p gpurun_out/r6d
timeout -k 10 500 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_c5.py tests/test_gpu_ring.py tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread > gpurun_out/r6d/tests.txt 2>&1
rc=$?
tail -25 gpurun_out/r6d/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "
import sys, json; sys.argv=['bench.py']
import bench
from flodbadd_amd import _native as N, synth
import ctypes as C
lib = N.gpu_lib()
cfg = N.FbConfig(); cfg.abi_version = N.FB_ABI_VERSION; cfg.filter = N.FB_FILTER_GLOBAL_ONLY
cfg.max_batch_packets = 1 << 20; cfg.flow_capacity = 1 << 21; cfg.flags = N.FB_CFG_FIXED_TABLE
ctx = C.c_void_p(lib.fb_create(0, C.byref(cfg)))
fr, of = synth.generate(2, 1 << 20)
print(json.dumps(bench.host_ring(N, lib, ctx, fr, of)))
" > gpurun_out/r6d/ring.json 2> gpurun_out/r6d/ring.err
tail -c 1500 gpurun_out/r6d/ring.json
