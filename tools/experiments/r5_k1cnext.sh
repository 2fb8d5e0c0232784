#!/bin/bash
# K1c next-group grab one group ahead and lazy table init (FB_COMB_NEXT, FB_COMB_LAZY_INIT; product: both)
# vs k1cold (neither): the GPU tests named in TESTS on the product, the per-workgroup K2 / K1c
# trace of both (flowtr / flowtr0), then the C4 line uniform and Zipf(1.1), interleaved
# (tools/build_variants.sh builds the variants).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest ${TESTS:-tests -m gpu} \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/k1cnext_tests.log 2>&1 || { tail -30 gpurun_out/k1cnext_tests.log; exit 1; }
tail -1 gpurun_out/k1cnext_tests.log
for v in ${TRVARS:-flowtr}; do
  echo "== trace $v"
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 200 python -u tools/experiments/flow_trace.py \
    > gpurun_out/flow_trace_$v.txt 2> gpurun_out/flow_trace_$v.err || { tail gpurun_out/flow_trace_$v.err; exit 1; }
  python - gpurun_out/flow_trace_$v.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); k = d["k2"]
    print(d["workload"], "flow_ms", d["flow_ms"], "K2 span", k["span_us"], "dur p50", k["dur_us"]["p50"], "max",
          k["dur_us"]["max"], "p99", k["dur_us"]["p99"], "K1c span", d.get("k1c", {}).get("span_us"), d.get("k1c", {}).get("phases_us"))
PY
done
for r in 1 2; do
  for v in product ${ABVARS:-k1cold}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for z in "" "--zipf 1.1"; do
      FLODBADD_GPU_LIB=$L timeout -k 10 200 python bench.py --config 4 $z --table-only --steps 20 --warmup 4 \
        --no-other-mode --no-cpu-baseline --no-host --no-imix --no-queue --no-copy-ref > gpurun_out/k1n.json 2> gpurun_out/k1n.err || { tail gpurun_out/k1n.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/k1n.json'));e=d['extra'];print('$v', '${z:-uniform}', d['value'], e['c4_sync']['value'], e['c4_stages']['flow_update_ms'])"
    done
  done
done
