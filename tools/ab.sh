#!/bin/bash
# A/B timing of variant libraries on chosen configs (GPU box):
#   tools/ab.sh "old ring1 ring4" "B_karman64k D_cube64"
# Each (variant, config) runs twice in its own process; prints one JSON line per run.
cd "$(dirname "$0")/.."
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for v in $1; do
    for c in $2; do
      echo -n "$v "
      WOS_LIB_PATH=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var/libwos_$v.so timeout -k 5 120 python3 tools/time_configs.py $c 2>/dev/null | tail -1
    done
  done
done
