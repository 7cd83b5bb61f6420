#!/bin/bash
# A/B timing of an environment switch on chosen configs (GPU box):
#   tools/ab_env.sh WOS_PHASES "1 2" "B_karman64k D_cube64"
# Each (value, config) runs ROUNDS times in its own process; prints one JSON line per run
# prefixed with the value (tools/ab_summary.py reads it).
cd "$(dirname "$0")/.."
VAR=$1
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for v in $2; do
    for c in $3; do
      echo -n "$VAR=$v "
      env "$VAR=$v" timeout -k 5 120 python3 tools/time_configs.py $c 2>/dev/null | tail -1
    done
  done
done
