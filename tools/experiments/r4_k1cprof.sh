#!/bin/bash
# Round 4: per-workgroup wall-clock phases of K1c k_flow_combine (device printf, timing-only variant
# var_k1cprof.so) in the C4 Zipf(1.1) one-stream table-only run.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4k1cp; rm -rf "$OUT"; mkdir -p "$OUT"
FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_k1cprof.so timeout -k 10 200 python3 bench.py --config 4 --zipf 1.1 --c4-sync --table-only --steps 1 --warmup 1 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/zipf.txt" 2> "$OUT/zipf.err" || exit 1
grep -c CP "$OUT/zipf.txt"
