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
# ALL=1: rebuild every object with the extra flags (needed when they change shared headers);
# REBUILD="dmf_trace ...": the objects to rebuild (default dmf_fuse)
REBUILD=${REBUILD:-dmf_fuse}
OBJS=""
for f in dmf_core dmf_trace dmf_fuse dmf_ogrid dmf_comm dmf_io; do
  if [[ " $REBUILD " == *" $f "* ]] || [ -n "$ALL" ]; then
    EXTRA=""; [ $f = dmf_fuse ] && EXTRA="-mllvm -amdgpu-atomic-optimizer-strategy=None"  # as the Makefile
    /opt/rocm/bin/hipcc $FLAGS $EXTRA "$@" -c csrc/$f.hip -o "$OUT/$f.o" &
    OBJS="$OBJS $OUT/$f.o"
  else
    OBJS="$OBJS build/$f.o"
  fi
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libdmf.so" $OBJS -Wl,-soname,libdmf.so -L/opt/rocm/lib -lrccl
echo "$OUT/libdmf.so"
