#!/bin/bash
# A/B timing of environment settings (GPU box, repo root):
#   tools/ab_modes.sh "A=0,B=1 A=1" "B_karman64k D_cube64"
# Each mode is a comma-separated list of VAR=value; each (mode, config) runs ROUNDS times
# in its own process; prints one JSON line per run prefixed with the mode.
cd "$(dirname "$0")/.."
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for m in $1; do
    for c in $2; do
      echo -n "$m "
      env ${m//,/ } timeout -k 5 120 python3 tools/time_configs.py $c 2>/dev/null | tail -1
    done
  done
done
