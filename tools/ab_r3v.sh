#!/bin/bash
# head windows (WOS_TASK_HEAD x WOS_TASK_GRAB_HEAD) of the task queues: bit-exactness (B, D), latency probe, configs C / D
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
for v in h0 h4x16; do
  for c in B D; do
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/h_${v}_$c.json $c --shard8 >> gpurun_out/r3v_dump.log 2>&1 || exit 1
  done
done
for c in B D; do
  python3 tools/dump_solution.py --compare gpurun_out/h_h0_$c.json gpurun_out/h_h4x16_$c.json >> gpurun_out/r3v_dump.log 2>&1 || exit 1
done
ROUNDS=2 timeout -k 10 800 bash tools/ab_latency.sh "h0 h1x32 h2x32 h1x16 h4x16 q8g32" > gpurun_out/r3v_ab.log 2>&1 &&
ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "h0 h1x32 h4x16" "C_dirichlet512 D_cube64" > gpurun_out/r3v_ab_cfg.log 2>&1
