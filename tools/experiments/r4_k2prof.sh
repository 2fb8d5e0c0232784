#!/bin/bash
# Round 4: per-workgroup wall-clock phases of K2 k_flow_apply (device printf, timing-only variant
# var_k2prof.so) in the C4 one-stream table-only run, uniform and Zipf(1.1).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4k2p; rm -rf "$OUT"; mkdir -p "$OUT"
for v in unif zipf; do
  Z=""; [ $v = zipf ] && Z="--zipf 1.1"
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_k2prof.so timeout -k 10 200 python3 bench.py --config 4 $Z --c4-sync --table-only --steps 1 --warmup 1 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/$v.txt" 2> "$OUT/$v.err" || exit 1
  grep -c KP "$OUT/$v.txt"
done
