#!/bin/bash
# Round 4: a second K1c launch (FB_COMB_HELP workgroups) on the update stream of the pipelined call,
# taking hot groups from the same counter as the main launch (FB_COMB_GRID workgroups on the parse
# stream) -- interleaved C4 pipelined table-only lines (Zipf(1.1) and uniform) per variant
# (tools/build_variants.sh: h0 = the product geometry), then the GPU tests of the pipelined and
# skewed paths with two helper variants loaded in place of the product library.
# The knob lives in commit 3636758 (reverted in 0fa2f08): build the variants from that tree.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4kh; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --no-copy-ref --table-only"
for rep in 1 2; do
  for v in ${VARS:-h0 g768h256 g512h512 g1024h512}; do
    for z in "--zipf 1.1" ""; do
      f=$OUT/pipe_${v}_${rep}${z:+z}.json
      step pipe env FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_$v.so timeout -k 10 300 python3 bench.py --config 4 $z --steps 20 --warmup 3 $X > "$f" 2> "$f.err"
      python3 -c "import json; d=json.loads(open('$f').readline()); print('$v rep $rep zipf=${z:+1}', d['value'], d['ms_per_step'])"
    done
  done
done
for v in g512h512 g768h256; do
  step tests_$v env FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_$v.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "async or zipf or hot or history or grow or c4 or combine" > "$OUT/tests_$v.log" 2>&1
  tail -1 "$OUT/tests_$v.log"
done
