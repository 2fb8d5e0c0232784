#!/bin/bash
# K2 / K1c same-slot wave folds (FB_K2_FOLD, FB_COMB_FOLD): the session-table tests on the product
# (folds on), the per-workgroup K2 / K1c trace with the folds on / off (flowtr / flowtr0), then the C4
# line uniform and Zipf(1.1) for the product vs nofold (both off) and k2only (K1c's off), interleaved
# (tools/build_variants.sh builds the variants beforehand).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_history.py tests/test_gpu_parity.py \
  tests/test_gpu_async.py tests/test_gpu_grow.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/k2fold_tests.log 2>&1 || { tail -30 gpurun_out/k2fold_tests.log; exit 1; }
tail -1 gpurun_out/k2fold_tests.log
for v in flowtr flowtr0; do
  echo "== trace $v"
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 200 python -u tools/experiments/flow_trace.py \
    > gpurun_out/flow_trace_$v.txt 2> gpurun_out/flow_trace_$v.err || { tail gpurun_out/flow_trace_$v.err; exit 1; }
  python - gpurun_out/flow_trace_$v.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); k = d["k2"]
    print(d["workload"], "flow_ms", d["flow_ms"], "K2 span", k["span_us"], "dur max", k["dur_us"]["max"],
          "p99", k["dur_us"]["p99"], "K1c span", d.get("k1c", {}).get("span_us"))
PY
done
for r in 1 2; do
  for v in product ${ABVARS:-nofold k2only}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for z in "" "--zipf 1.1"; do
      FLODBADD_GPU_LIB=$L timeout -k 10 200 python bench.py --config 4 $z --table-only --steps 20 --warmup 4 \
        --no-other-mode --no-cpu-baseline --no-host --no-imix --no-queue --no-copy-ref > gpurun_out/k2f.json 2> gpurun_out/k2f.err || { tail gpurun_out/k2f.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/k2f.json'));e=d['extra'];print('$v', '${z:-uniform}', d['value'], e['c4_sync']['value'], e['c4_stages']['flow_update_ms'])"
    done
  done
done
