#!/bin/bash
# C2 kernel time per launch vs batches per launch on one box (fixed per-launch cost), two rounds.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --rotate 32"
for r in 1 2; do
  for b in 2 4 8 16 24 32; do
    timeout -k 10 120 python bench.py --steps 96 --warmup 32 --batches-per-launch $b $X > gpurun_out/bf.json 2>gpurun_out/bf.err || { tail gpurun_out/bf.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bf.json'));r=d['roofline'];print('bpl=$b', d['value'], r['kernel_ms_per_launch'], round(r['kernel_ms_per_launch']*1e3/$b,2))"
  done
done
