# Combine-threshold sweep (k_flow_combine) on C4 Zipf(1.1), interleaved, + a kernel-trace profile.
mkdir -p gpurun_out/sweepc
set -e
for r in 1 2; do
for v in s256g1024cm48 s128g2048cm48 s256g1024cm64 s128g2048cm32; do
  FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 150 python bench.py --config 4 --zipf 1.1 --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > gpurun_out/sweepc/$v.$r.json 2> gpurun_out/sweepc/$v.$r.err
  echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/sweepc/$v.$r.json').read().strip().splitlines()[-1]);print(d['value'],d['extra']['c4_stages']['flow_update_ms'])")"
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_s128g2048cm48.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweepc/prof -o zipf -- python bench.py --config 4 --zipf 1.1 --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > gpurun_out/sweepc/prof.log 2>&1
