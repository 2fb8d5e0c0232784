#!/bin/bash
# Round 4, first GPU pass at HEAD: GPU tests, the driver's default bench line, a 2-rank launch
# through bench.py's own spawner (both ranks on the one GPU, C5 exchange over gloo), the driver's
# exact command under a kernel trace (its bench line kept beside the trace), and separate
# FETCH_SIZE / WRITE_SIZE passes for the C2 / C3 / C4 dominant kernels.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4a; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/gputests.log" 2>&1
tail -3 "$OUT/gputests.log"
step bench timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step bench_w2 env FB_C5_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  > "$OUT/bench_w2.json" 2> "$OUT/bench_w2.err"
cd /tmp
step drvprof timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/drv" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
  > "$OUT/drv_bench.json" 2> "$OUT/drv_bench.err"
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --no-c4"
for c in 2 3; do
  step pmc_f$c timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c$c" -o run -- python3 "$R/bench.py" --config $c --steps 32 --warmup 32 $X > "$OUT/pmc_fetch_c$c.json" 2>&1
  step pmc_w$c timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_c$c" -o run -- python3 "$R/bench.py" --config $c --steps 32 --warmup 32 $X > "$OUT/pmc_write_c$c.json" 2>&1
done
step pmc_f4 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c4" -o run -- python3 "$R/bench.py" --config 4 --c4-sync --table-only --steps 8 --warmup 4 $X > "$OUT/pmc_fetch_c4.json" 2>&1
step pmc_w4 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_c4" -o run -- python3 "$R/bench.py" --config 4 --c4-sync --table-only --steps 8 --warmup 4 $X > "$OUT/pmc_write_c4.json" 2>&1
du -sh "$OUT"/* >&2
