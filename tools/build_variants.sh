#!/bin/bash
# Build experimental variants of libflodbadd_gpu.so (not product): VARIANTS="name:-DFLAG=..,-DFLAG2 ..."
# -> flodbadd_amd/build/var_<name>.so, loaded by setting FLODBADD_GPU_LIB.
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
for v in $VARIANTS; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr ',' ' ')
  objs=""
  for s in fb_parse fb_compact fb_flow fb_hist fb_capi fb_ring fb_enrich fb_dns; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -Iinclude -c flodbadd_amd/csrc/$s.hip \
      -o flodbadd_amd/build/var_${name}_$s.o &
    objs="$objs flodbadd_amd/build/var_${name}_$s.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o flodbadd_amd/build/var_$name.so $objs
  rm -f $objs
done
