#!/bin/bash
# Build an A/B experiment library from the working copy of csrc/dmf_fuse.hip into
# depth-map-fusion-utils_amd/build_exp/<name>/libdmf.so (the other objects come from build/).
# Run with DMF_LIB=<that path>.  Extra hipcc flags: $2...
set -e
cd "$(dirname "$0")/../depth-map-fusion-utils_amd"
NAME=$1; shift
OUT=build_exp/$NAME
mkdir -p "$OUT"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -Wall -Wno-unused-function -I../include -Icsrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c csrc/dmf_fuse.hip -o "$OUT/dmf_fuse.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libdmf.so" build/dmf_core.o build/dmf_trace.o "$OUT/dmf_fuse.o" build/dmf_ogrid.o -Wl,-soname,libdmf.so
echo "$OUT/libdmf.so"
