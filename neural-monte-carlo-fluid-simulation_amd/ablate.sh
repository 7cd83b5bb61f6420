#!/bin/bash
# Timing-only ablation builds (wrong results by construction; never shipped).
set -e
mkdir -p build/abl lib/abl
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w"
hipcc $FLAGS -c csrc/wos_capi.hip -o build/abl/capi.o
hipcc $FLAGS -x hip -c csrc/wos_host_scene.cpp -o build/abl/scene.o
for v in "base:" "nosil:-DWOS_ABL_NO_SIL=1" "noray:-DWOS_ABL_NO_RAY=1" "onerej:-DWOS_ABL_ONE_REJ=1" "nostats:-DWOS_ABL_NO_STATS=1" "geomoff:-DWOS_ABL_NO_SIL=1 -DWOS_ABL_NO_RAY=1"; do
  name=${v%%:*}; defs=${v#*:}
  hipcc $FLAGS $defs -c csrc/wos_kernel.hip -o build/abl/k_$name.o &
done
wait
for v in base nosil noray onerej nostats geomoff; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o lib/abl/libwos_$v.so build/abl/k_$v.o build/abl/capi.o build/abl/scene.o
done
