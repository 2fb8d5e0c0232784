#!/bin/bash
# Build tools/ubench_ws_<variant> (role-specialised parse kernel timing + stamps; not product).
# VARIANTS: space-separated load:u:store:lb:win geometries (loader waves : tiles per loader wave :
# storer waves : look-back waves : LDS slots : header prefetch depth), default the product geometry.
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
gcc -O2 -fopenmp -fPIC -c flodbadd_amd/csrc/fb_synth.c -o flodbadd_amd/build/fb_synth_ub.o
for v in ${VARIANTS:-8:1:4:2:5:3}; do
  IFS=: read -r l u st lb sl dp <<< "$v"
  tag=${l}_${u}_${st}_${lb}_${sl}_${dp}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFB_WS_LOAD=$l -DFB_WS_U=$u -DFB_WS_STORE=$st \
    -DFB_WS_LB=$lb -DFB_WS_SLOTS=$sl -DFB_WS_DEPTH=$dp ${EXTRA:-} -Iinclude -c tools/ubench_ws.hip -o flodbadd_amd/build/ubench_ws_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 flodbadd_amd/build/ubench_ws_$tag.o flodbadd_amd/build/fb_synth_ub.o \
    -fopenmp -lm -o tools/ubench_ws_$tag
done
