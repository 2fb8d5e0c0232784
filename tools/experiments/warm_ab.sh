#!/bin/bash
# C2 headline at the driver's settings (--steps 20) with warmup 5 vs 32, interleaved, extras off.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch"
for r in 1 2 3; do
  for w in 5 32; do
    timeout -k 10 120 python bench.py --steps 20 --warmup $w $X > gpurun_out/wab_$w.json 2>gpurun_out/wab.err || { tail gpurun_out/wab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/wab_$w.json'));print('w=$w', d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['timed_region_host_us_outside_kernels'])"
  done
done
