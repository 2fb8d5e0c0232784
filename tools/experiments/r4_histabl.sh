#!/bin/bash
# Round 4: where the C4 Zipf(1.1) history's slow-list kernel goes -- timing-only ablation builds of
# fb_hist.hip (tools/build_variants.sh: nowalk / nosort / noload) against the product, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4ha; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
cd /tmp
for v in product nowalk nosort noshort noload; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --table-only --steps 4 --warmup 2 $X > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  echo "== $v done"
done
