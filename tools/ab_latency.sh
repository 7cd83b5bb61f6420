#!/bin/bash
# A/B of variant libraries on the latency probe (GPU box):
#   tools/ab_latency.sh "base cell0 ray0" > gpurun_out/x.log
# Each variant runs ROUNDS times (default 2) in its own process, interleaved.
cd "$(dirname "$0")/.."
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for v in $1; do
    WOS_LIB_PATH=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var/libwos_$v.so timeout -k 5 120 python3 tools/latency_probe.py 2>/dev/null | sed "s/^/$v /" || exit 1
  done
done
