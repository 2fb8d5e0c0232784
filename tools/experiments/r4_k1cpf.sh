#!/bin/bash
# Round 4: K1c fetching the next hot group while finishing the current one (commit 4da7e0a, built as
# the product library; reverted in 09ef277) -- every GPU test, then interleaved A/B against the
# previous HEAD (var_base.so: VARIANTS="base:-DFB_NOP" tools/build_variants.sh): C4 Zipf(1.1) one-stream kernel traces
# and pipelined table-only lines.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4pf; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputests.log" 2>&1
tail -1 "$OUT/gputests.log"
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only"
for v in base new; do
  L=$R/flodbadd_amd/libflodbadd_gpu.so; [ $v = base ] && L=$R/flodbadd_amd/build/var_base.so
  cd /tmp
  step tr_$v env FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --steps 10 --warmup 2 $X > "$OUT/tr_$v.json" 2> "$OUT/tr_$v.err"
  cd "$R"
done
for rep in 1 2; do
  for v in base new; do
    L=$R/flodbadd_amd/libflodbadd_gpu.so; [ $v = base ] && L=$R/flodbadd_amd/build/var_base.so
    for z in "--zipf 1.1" ""; do
      f=$OUT/pipe_${v}_${rep}${z:+z}.json
      step pipe env FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 python3 bench.py --config 4 $z --steps 20 --warmup 3 $X > "$f" 2> "$f.err"
      python3 -c "import json; d=json.loads(open('$f').readline()); print('$v rep $rep zipf=${z:+1}', d['value'], d['ms_per_step'])"
    done
  done
done
