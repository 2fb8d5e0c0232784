#!/bin/bash
# Dense-mode C2 under a kernel trace (k_parse_dense), extras off; then C3 at 12 vs 32 batches per launch.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/profdense; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --mode dense --steps 100 --warmup 10 $X > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cd "$R"
for r in 1 2; do for rot in 12 32; do
  timeout -k 10 200 python bench.py --config 3 --rotate $rot --steps 96 --warmup 24 $X > gpurun_out/c3r.json 2>gpurun_out/c3r.err || { tail gpurun_out/c3r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c3r.json'));print('C3 rotate $rot', d['value'], d['roofline']['frac'])"
done; done
