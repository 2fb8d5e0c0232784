#!/bin/bash
# Round 4: SQ counters (one --pmc pass) of the C4 Zipf(1.1) one-stream table-only run: where the
# K1c / K2 waves spend their cycles.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4k1cpmc; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$OUT/sq" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --table-only --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > "$OUT/sq.json" 2> "$OUT/sq.err" || { tail -5 "$OUT/sq.err"; exit 1; }
echo done
