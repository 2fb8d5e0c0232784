#!/bin/bash
# Round-2 profiles at HEAD: C2/C3/C4 bench + kernel trace + FETCH/WRITE passes (tools/experiments/r2_profile.sh),
# the driver's C2 command under a kernel trace (tools/prof_driver.sh), and a dense-mode C2 trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd)
bash tools/experiments/r2_profile.sh || exit 1
bash tools/prof_driver.sh || exit 1
OUT=$R/gpurun_out/profdense; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --mode dense --steps 100 --warmup 10 \
  --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
tail -c 300 "$OUT/bench.json"
