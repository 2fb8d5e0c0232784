#!/bin/bash
# C4 Zipf one-stream history time: product vs timing variants (tools/build_variants.sh).
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for v in ${ZVARS:-product}; do
  if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config 4 --c4-sync --zipf 1.1 --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > gpurun_out/zv.json 2> gpurun_out/zv.err || { tail -5 gpurun_out/zv.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/zv.json'));e=d['extra']['c4_stages'];print('$v', d['value'], 'history_ms', e['history_ms'], e['history_chars'])"
done
