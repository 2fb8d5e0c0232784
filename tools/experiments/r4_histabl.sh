#!/bin/bash
# Round 4: where the C4 Zipf(1.1) history's slow-list kernel goes -- timing-only ablation builds of
# fb_hist.hip (tools/build_variants.sh: nowalk / nosort / noload) against the product, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4ha; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
cd /tmp
for v in product nowalk nosort noload; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --table-only --steps 4 --warmup 2 $X > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  echo "== $v done"
done
# dense (batch-wide) output vs batch size: per-launch vs per-round costs
cd "$R"
for n in 1048576 4194304; do
  timeout -k 10 200 python3 bench.py --config 2 --mode dense --packets $n --rotate 8 --steps 16 --warmup 4 --no-c4 --no-imix --no-other-mode --no-single-launch --no-host --no-cpu-baseline > "$OUT/dense_$n.json" 2> "$OUT/dense_$n.err" || exit 1
  timeout -k 10 200 python3 bench.py --config 2 --packets $n --rotate 8 --batches-per-launch 1 --steps 16 --warmup 4 --no-c4 --no-imix --no-other-mode --no-single-launch --no-host --no-cpu-baseline > "$OUT/seg1_$n.json" 2> "$OUT/seg1_$n.err" || exit 1
  echo "== dense / seg $n done"
done
