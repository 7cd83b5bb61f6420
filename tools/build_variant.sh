#!/bin/bash
# Builds a variant of the engine library for A/B timing or diagnostics (never shipped):
#   tools/build_variant.sh NAME "-DWOS_DIAG=1 ..."   ->  neural-monte-carlo-fluid-simulation_amd/lib/var/libwos_NAME.so
# Select it at run time with WOS_LIB_PATH (tools/time_variants.py does).
set -e
cd "$(dirname "$0")/../neural-monte-carlo-fluid-simulation_amd"
NAME=$1; DEFS=$2
SRC=${WOS_VARIANT_SRC:-csrc}  # an experimental copy of the sources (the shipped csrc/ stays untouched)
mkdir -p build/var lib/var
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w $DEFS"
hipcc $FLAGS -c $SRC/wos_kernel.hip -o build/var/k_$NAME.o &
hipcc $FLAGS -c $SRC/wos_bvc.hip -o build/var/b_$NAME.o &
hipcc $FLAGS -c $SRC/wos_robust.hip -o build/var/r_$NAME.o &
hipcc $FLAGS -c $SRC/wos_capi.hip -o build/var/c_$NAME.o &
hipcc $FLAGS -x hip -c $SRC/wos_host_scene.cpp -o build/var/s_$NAME.o &
hipcc $FLAGS -x hip -c $SRC/wos_bvc_host.cpp -o build/var/h_$NAME.o &
hipcc $FLAGS -x hip -c $SRC/wos_fcpw_bvh.cpp -o build/var/t_$NAME.o &
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o lib/var/libwos_$NAME.so build/var/k_$NAME.o build/var/b_$NAME.o build/var/r_$NAME.o \
  build/var/c_$NAME.o build/var/s_$NAME.o build/var/h_$NAME.o build/var/t_$NAME.o
echo lib/var/libwos_$NAME.so
