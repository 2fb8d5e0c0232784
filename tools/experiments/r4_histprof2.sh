#!/bin/bash
# Round 4: per-(partition, block) wall-clock stamps (device printf, timing-only variant
# var_prof2.so) of the split history kernels under the C4 Zipf(1.1) batch, and the timer's rate.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4hp2; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 60 python3 -c "
import ctypes; h = ctypes.CDLL('libamdhip64.so'); v = ctypes.c_int()
print('wall clock kHz', h.hipDeviceGetAttribute(ctypes.byref(v), 10017, 0), v.value)" > "$OUT/rate.txt" 2>&1
FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_prof2.so timeout -k 10 200 python3 bench.py --config 4 --zipf 1.1 --c4-sync --table-only --steps 1 --warmup 1 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/out.txt" 2> "$OUT/err.txt"
rc=$?; cat "$OUT/rate.txt"; grep -c HP2 "$OUT/out.txt"; exit $rc
