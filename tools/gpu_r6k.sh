#!/bin/bash
# shared queue + table: blocks on CUs / DIV (product DIV 4; variants 1, 2, 8), interleaved (second sweep: 8, 16, 32, 64)
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6k2; mkdir -p "$OUT"; export TMPDIR=/tmp
#timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
#tail -1
for rep in 1 2; do
for v in qs8 qs16 qs32 qs64; do
  L=$R/flodbadd_amd/build/var_$v.so; [ $v = cur ] && L=$R/flodbadd_amd/libflodbadd_gpu.so
  echo -n "$v: "; FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/queue_table_prof.py 60 > "$OUT/$v.$rep.log" 2>&1 || { tail "$OUT/$v.$rep.log"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/$v.$rep.log').read().splitlines()[-1]);print(d['value'],d['ms_per_batch'])"
done; done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/qt" -o run -- python3 "$R/tools/queue_table_prof.py" 40 > "$OUT/qt.log" 2>&1 || { tail "$OUT/qt.log"; exit 1; }
