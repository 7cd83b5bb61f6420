#!/bin/bash
# Generic A/B (GPU box): every variant against the first one -- solution hashes on configs
# B, C and D (B and D with their stride-8 shards; must be identical), then the latency probe
# and the config timings, ROUNDS interleaved runs each.
#   tools/ab_generic.sh TAG "base v1 v2" [probe-only case]
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
TAG=$1; VARS=$2
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
REF=${VARS%% *}
for v in $VARS; do
  for c in B C D; do
    sh8=""; [ $c != C ] && sh8="--shard8"
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/${TAG}_d_${v}_$c.json $c $sh8 >> gpurun_out/${TAG}_dump.log 2>&1 || exit 1
  done
done
for v in $VARS; do
  [ $v = $REF ] && continue
  for c in B C D; do
    python3 tools/dump_solution.py --compare gpurun_out/${TAG}_d_${REF}_$c.json gpurun_out/${TAG}_d_${v}_$c.json >> gpurun_out/${TAG}_dump.log 2>&1 || { echo "NOT BIT-EXACT: $v $c"; exit 1; }
  done
done
echo "bit-exact: $VARS"
ROUNDS=${ROUNDS:-2} timeout -k 10 700 bash tools/ab_latency.sh "$VARS" > gpurun_out/${TAG}_ab.log 2>&1 &&
ROUNDS=${ROUNDS:-2} timeout -k 10 400 bash tools/ab.sh "$VARS" "C_dirichlet512 D_cube64" > gpurun_out/${TAG}_ab_cfg.log 2>&1
