#!/bin/bash
# C4 (one stream, records and table-only) for the product and timing-only variants (tools/build_variants.sh).
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
for r in 1 2; do
  for v in ${CVARS:-product}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for t in "" "--table-only"; do
      FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config 4 --steps 20 --warmup 3 $X $t > gpurun_out/c4v.json 2> gpurun_out/c4v.err || { tail -5 gpurun_out/c4v.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/c4v.json'));e=d['extra'];print('$v C4 $t', d['value'], e['c4_stages']['parse_ms'], e['c4_stages']['flow_update_ms'], e['c4_sync']['value'])"
    done
  done
done
