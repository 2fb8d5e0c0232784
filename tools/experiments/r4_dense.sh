#!/bin/bash
# Round 4: dense output with dynamic tile hand-out -- GPU dense / compact / parity tests, then the
# C2 / C3 dense bench lines and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4dn2; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_dense.py -x -v --timeout 60 --timeout-method thread > "$OUT/dense_tests.log" 2>&1 || { tail -30 "$OUT/dense_tests.log"; exit 1; }
tail -1 "$OUT/dense_tests.log"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
X="--mode dense --steps 200 --warmup 20 --no-c4 --no-imix --no-other-mode --no-single-launch --no-host --no-cpu-baseline"
for c in 2 3; do
  timeout -k 10 200 python3 bench.py --config $c $X > "$OUT/dense_c$c.json" 2> "$OUT/dense_c$c.err" || { tail -3 "$OUT/dense_c$c.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/dense_c$c.json').readline()); print('dense C$c', d['value'], d['ms_per_step'])"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --config 2 $X > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -3 "$OUT/trace.err"; exit 1; }
echo done
