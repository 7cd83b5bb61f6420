#!/bin/bash
# Register / scratch / occupancy of the engine kernels (compile only, no GPU):
#   tools/kres.sh ["-DMACRO=..."]
cd "$(dirname "$0")/../neural-monte-carlo-fluid-simulation_amd"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w $1 -c csrc/wos_kernel.hip \
  -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name/ {n=$NF; sub(/\[.*/,"",n); name=$0; sub(/.*Function Name: /,"",name); sub(/ \[.*/,"",name)}
       /VGPRs: / {v=$4} /TotalSGPRs/ {s=$4} /ScratchSize/ {sc=$5}
       /Occupancy/ {o=$5; if (name ~ /walk|first_ball/) printf "%-52s VGPR %4s SGPR %4s scratch %4s occ %s\n", substr(name,9,48), v, s, sc, o}'
