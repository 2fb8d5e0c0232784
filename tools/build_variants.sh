#!/bin/bash
# Build experimental (timing-only) variants of libflodbadd_gpu.so -- never the product.
#   VARIANTS="name:-DFLAG=..,-DFLAG2 ..."   compile-time knobs of the product sources
#   PATCH_<name>="python expression"       optional source edit applied to a COPY of csrc/ for
#                                          variant <name> (ablations live here, not in csrc/):
#                                          a python snippet run with `s` = file text, `f` = file name
# -> flodbadd_amd/build/var_<name>.so, loaded by setting FLODBADD_GPU_LIB.
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
for v in $VARIANTS; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr ',' ' ')
  src=flodbadd_amd/csrc
  pvar="PATCH_${name}"
  if [ -n "${!pvar:-}" ]; then
    tmp=$(mktemp -d); mkdir -p $tmp/pkg; cp -r flodbadd_amd/csrc $tmp/pkg/csrc; ln -s $(pwd)/include $tmp/include
    src=$tmp/pkg/csrc
    PATCH="${!pvar}" python3 - $src <<'PY'
import glob, os, sys
code = os.environ["PATCH"]
for f in glob.glob(sys.argv[1] + "/*.hip") + glob.glob(sys.argv[1] + "/*.h"):
    s = open(f).read()
    loc = {"s": s, "f": os.path.basename(f)}
    exec(code, {}, loc)
    if loc["s"] != s:
        open(f, "w").write(loc["s"])
        print("patched", os.path.basename(f))
PY
  fi
  objs=""
  for s in $(python3 -c "import sys; sys.path.insert(0, \"flodbadd_amd\"); import build; print(\" \".join(x[:-4] for x in build.HIP_SOURCES))"); do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -Iinclude -I$src -c $src/$s.hip \
      -o flodbadd_amd/build/var_${name}_$s.o &
    objs="$objs flodbadd_amd/build/var_${name}_$s.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o flodbadd_amd/build/var_$name.so $objs
  rm -f $objs
done
