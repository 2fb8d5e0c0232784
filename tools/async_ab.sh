cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/aab
for r in 1 2; do for d in 1 2 3; do
  FB_ASYNC_PARSE_GRID_DIV=$d timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 4 --no-cpu-baseline --no-other-mode > gpurun_out/aab/d$d.$r.json 2>gpurun_out/aab/d$d.$r.err || { tail -3 gpurun_out/aab/d$d.$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/aab/d$d.$r.json'));print('div $d', d['value'], d['extra']['c4_sync']['value'])"
done; done
