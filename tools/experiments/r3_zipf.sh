#!/bin/bash
# C4 with Zipf(1.1) flow popularity as the main line (pipelined; table-only and records), plus the
# config-4 extras (one-stream Zipf line, dense output with the table).
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
X="--no-cpu-baseline --no-host --no-imix --no-single-launch"
for t in "--table-only" ""; do
  timeout -k 10 300 python3 bench.py --config 4 --zipf 1.1 --steps 20 --warmup 3 $X $t > gpurun_out/zipf.json 2> gpurun_out/zipf.err || { tail -5 gpurun_out/zipf.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/zipf.json'));e=d['extra'];print('zipf $t', d['value'], e['c4_stages']['parse_ms'], e['c4_stages']['flow_update_ms'], 'sync', e['c4_sync']['value'], 'zipf-extra', e.get('c4_zipf'), 'dense', e.get('mode_dense',{}).get('value'))"
done
