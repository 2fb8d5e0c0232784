#!/bin/bash
# GPU box: per config (C2 C3 C4) the bench line, a kernel-trace --stats run and separate
# FETCH_SIZE / WRITE_SIZE --pmc passes (never combined with tracing), each step time-limited.
# Steps are whole launches (C2 32 batches per launch, C3 12, C4 1) so per-launch PMC medians are
# comparable.  Summarise locally afterwards with tools/prof_summary.py.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/prof; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { "$@"; rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
for CFG in ${CFGS:-2 3 4}; do
  case $CFG in
    2) W=32; ST=96; SP=64;;
    3) W=12; ST=96; SP=48;;
    4) W=2; ST=10; SP=6;;
  esac
  NO="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch"
  step timeout -k 10 300 python3 bench.py --config $CFG --steps 200 --warmup 20 > "$OUT/bench_c$CFG.json" 2> "$OUT/bench_c$CFG.err"
  cd /tmp
  step timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps $ST --warmup $W $NO > "$OUT/trace_c$CFG.log" 2>&1
  step timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps $SP --warmup $W $NO > "$OUT/pmc_fetch_c$CFG.log" 2>&1
  step timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps $SP --warmup $W $NO > "$OUT/pmc_write_c$CFG.log" 2>&1
  cd "$R"
  echo "c$CFG done: $(head -c 300 $OUT/bench_c$CFG.json)"
done
