#!/bin/bash
# Round 5: k_parse_seg with cross-block chunk hand-out -- every GPU test, then the headline line
# (20 batches per launch) and the one-batch-per-launch line, product vs the static-share build
# (FB_SEG_DYN=0), interleaved, then the per-block trace of the product's hand-out.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5dyn${TAG:-}; rm -rf "$OUT"; mkdir -p "$OUT"
if [ -z "${NOTESTS:-}" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputests.log" 2>&1 || { echo "GPU tests failed"; grep -E "FAILED|Error|error" "$OUT/gputests.log" | head -20; tail -5 "$OUT/gputests.log"; exit 1; }
tail -1 "$OUT/gputests.log"
fi
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-c4 --no-copy-ref --no-queue"
for rep in 1 2; do
  for v in product static; do
    L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
    FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py $X > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { tail -3 "$OUT/$v.$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$v.$rep.json').readline()); print('$v', d['value'], d['roofline']['frac'], 'single', d['extra']['single_batch_launch']['value'])"
  done
done
FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_segtr.so timeout -k 10 120 python3 tools/experiments/seg_trace.py > "$OUT/trace.txt" 2>&1 || { tail -5 "$OUT/trace.txt"; exit 1; }
cat "$OUT/trace.txt"
