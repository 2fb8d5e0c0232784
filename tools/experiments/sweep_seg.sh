# Seg-kernel geometry sweep over prebuilt variants (tools/build_variants.sh), interleaved rounds.
mkdir -p gpurun_out/sweep
set -e
for r in ${SWEEP_ROUNDS:-1 2}; do
for v in ${SWEEP_VARIANTS:-w16b1 w12b2 w8b3 w8b4}; do
  FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 150 python bench.py --steps 400 --warmup 24 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > gpurun_out/sweep/$v.$r.json 2> gpurun_out/sweep/$v.$r.err
  echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/sweep/$v.$r.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'])")"
done
done
