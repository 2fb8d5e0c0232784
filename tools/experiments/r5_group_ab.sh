#!/bin/bash
# Round 5: grouped-unit group size (FB_GRP_UNITS variants) vs per-segment units, the C4 line, interleaved.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5grpab; rm -rf "$OUT"; mkdir -p "$OUT"
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --no-queue --no-copy-ref"
for rep in 1 2; do
  for v in off product g224 g160; do
    L=""; G=1; [ $v = off ] && G=0; [ $v != off ] && [ $v != product ] && L=$R/flodbadd_amd/build/var_$v.so
    FB_UNIT_GROUP=$G FLODBADD_GPU_LIB=$L timeout -k 10 300 python3 bench.py $X > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { tail -3 "$OUT/$v.$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$v.$rep.json').readline()); print('$v', d['extra']['c4']['value'])"
  done
done
