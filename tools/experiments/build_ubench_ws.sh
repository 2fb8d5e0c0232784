#!/bin/bash
# Build tools/ubench_ws_<variant> (segmented parse kernel timing + stamps; not product).
# VARIANTS: space-separated waves:blocks_per_cu geometries of k_parse_seg, default the product one.
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
gcc -O2 -fopenmp -fPIC -c flodbadd_amd/csrc/fb_synth.c -o flodbadd_amd/build/fb_synth_ub.o
for v in ${VARIANTS:-8:3}; do
  IFS=: read -r w bpc <<< "$v"
  tag=${w}_${bpc}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFB_SEG_WAVES=$w -DFB_SEG_BPC=$bpc ${EXTRA:-} -Iinclude \
    -c tools/experiments/ubench_ws.hip -o flodbadd_amd/build/ubench_ws_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 flodbadd_amd/build/ubench_ws_$tag.o flodbadd_amd/build/fb_synth_ub.o \
    -fopenmp -lm -o tools/ubench_ws_$tag
done
