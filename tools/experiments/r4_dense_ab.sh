#!/bin/bash
# Round 4: dense output (C2, 1M frames) -- product vs timing-only ablations, interleaved.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4dn; rm -rf "$OUT"; mkdir -p "$OUT"
X="--mode dense --steps 200 --warmup 20 --no-c4 --no-imix --no-other-mode --no-single-launch --no-host --no-cpu-baseline"
for rep in 1 2; do
  for v in product ${VARS:?timing variants to compare}; do
    L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
    FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py $X > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { tail -3 "$OUT/$v.$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$v.$rep.json').readline()); print('$v', d['value'], d['ms_per_step'])"
  done
done
