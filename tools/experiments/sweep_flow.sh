# C4 session-table sweep over prebuilt variants (tools/build_variants.sh), interleaved rounds:
# SWEEP_VARIANTS="a b" [SWEEP_ROUNDS="1 2"] [ZIPF=1.1] bash tools/experiments/sweep_flow.sh
mkdir -p gpurun_out/sweepf
set -e
Z=""; [ -n "${ZIPF:-}" ] && Z="--zipf $ZIPF"
for r in ${SWEEP_ROUNDS:-1 2}; do
for v in $SWEEP_VARIANTS; do
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 150 python bench.py --config 4 $Z --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > gpurun_out/sweepf/$v.$r.json 2> gpurun_out/sweepf/$v.$r.err
  echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/sweepf/$v.$r.json').read().strip().splitlines()[-1]);s=d['extra']['c4_stages'];print(d['value'],s['flow_update_ms'],s['parse_ms'],s.get('enrich_ms'),s.get('dns_parse_ms'),'hist',s.get('history_ms'))")"
done
done
