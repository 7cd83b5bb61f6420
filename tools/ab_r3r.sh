#!/bin/bash
# solo rejection sampler: bit-exactness (B with its stride-8 shard, 3D config D) and latency A/B
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
for v in s0 s4; do
  for c in B D; do
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/d_${v}_$c.json $c --shard8 >> gpurun_out/r3r_dump.log 2>&1 || exit 1
  done
done
for c in B D; do
  python3 tools/dump_solution.py --compare gpurun_out/d_s0_$c.json gpurun_out/d_s4_$c.json >> gpurun_out/r3r_dump.log 2>&1 || exit 1
done
ROUNDS=2 timeout -k 10 600 bash tools/ab_latency.sh "s0 s1 s2 s4" > gpurun_out/r3r_ab.log 2>&1
