#!/bin/bash
# Build tools/ubench_parse (ablation microbenchmark; not part of the product).
set -e
cd "$(dirname "$0")/.."
mkdir -p flodbadd_amd/build
gcc -O2 -fopenmp -fPIC -c flodbadd_amd/csrc/fb_synth.c -o flodbadd_amd/build/fb_synth_ub.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -c tools/ubench_parse.hip -o flodbadd_amd/build/ubench_parse.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 flodbadd_amd/build/ubench_parse.o flodbadd_amd/build/fb_synth_ub.o -fopenmp -lm -o tools/ubench_parse
