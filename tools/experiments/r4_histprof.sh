#!/bin/bash
# Round 4: per-phase wall-clock stamps (device printf, timing-only variant var_prof.so) of the
# history's slow-list workgroups under the C4 Zipf(1.1) batch.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4hp; rm -rf "$OUT"; mkdir -p "$OUT"
FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_prof.so timeout -k 10 200 python3 bench.py --config 4 --zipf 1.1 --c4-sync --table-only --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/out.txt" 2> "$OUT/err.txt"
rc=$?; grep -c HPROF "$OUT/out.txt"; exit $rc
