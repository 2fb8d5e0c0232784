#!/bin/bash
# Round 4, final GPU pass at HEAD: every GPU test, smoke(), the driver's default bench line, the
# driver's exact command under a kernel trace (its bench line beside it), and the C4 Zipf(1.1)
# pipelined table-only line.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4f; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/gputests.log" 2>&1
tail -3 "$OUT/gputests.log"
step smoke timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step bench timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
cd /tmp
step drvprof timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/drv" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
  > "$OUT/drv_bench.json" 2> "$OUT/drv_bench.err"
cd "$R"
step zipf timeout -k 10 300 python3 bench.py --config 4 --zipf 1.1 --table-only --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/zipf.json" 2> "$OUT/zipf.err"
du -sh "$OUT"/* >&2
