#!/bin/bash
# Build tools/ubench_parse_<threads>_u<tiles> (ablation microbenchmark; not part of the product).
# Variants are block threads:tiles per wave; the control-wave pipeline experiment
# (tools/parse_experiments.hip) is compiled in with FB_FRAME_WAVES = threads/64 - 1.
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
gcc -O2 -fopenmp -fPIC -c flodbadd_amd/csrc/fb_synth.c -o flodbadd_amd/build/fb_synth_ub.o
for v in ${VARIANTS:-512:2}; do
  t=${v%%:*}; u=${v##*:}; fw=$((t / 64 - 1))
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFB_BLOCK_THREADS=$t -DFB_UNIT_TILES=$u -DFB_FRAME_WAVES=$fw \
    -Iinclude -c tools/ubench_parse.hip -o flodbadd_amd/build/ubench_parse_${t}_u$u.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 flodbadd_amd/build/ubench_parse_${t}_u$u.o flodbadd_amd/build/fb_synth_ub.o \
    -fopenmp -lm -o tools/ubench_parse_${t}_u$u
done
