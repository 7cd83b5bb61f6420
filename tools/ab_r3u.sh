#!/bin/bash
# task queues (WOS_TASK_QUEUES) x window (WOS_TASK_GRAB): bit-exactness on B/D, latency probe, configs C / D
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
for v in q1g128 q8g64; do
  for c in B D; do
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/h_${v}_$c.json $c --shard8 >> gpurun_out/r3u_dump.log 2>&1 || exit 1
  done
done
for c in B D; do
  python3 tools/dump_solution.py --compare gpurun_out/h_q1g128_$c.json gpurun_out/h_q8g64_$c.json >> gpurun_out/r3u_dump.log 2>&1 || exit 1
done
ROUNDS=2 timeout -k 10 700 bash tools/ab_latency.sh "q1g128 q8g64 q8g128 q8g32 q1g64" > gpurun_out/r3u_ab.log 2>&1 &&
ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "q1g128 q8g64 q8g32" "C_dirichlet512 D_cube64" > gpurun_out/r3u_ab_cfg.log 2>&1
