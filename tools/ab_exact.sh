#!/bin/bash
# A/B of variant libraries (GPU box, repo root): solution hashes on B, D, C must equal the first
# variant's (DUMP="B D C E" to change the list), then ROUNDS interleaved timings on the named cases (tools/time_configs.py names).
#   tools/ab_exact.sh TAG "base v1 v2" ["B_karman64k C_dirichlet512 D_cube64"]
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1; VARS=$2; CFGS=${3:-"B_karman64k C_dirichlet512 D_cube64"}
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
REF=${VARS%% *}
for v in $VARS; do for c in ${DUMP:-B D C}; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 200 python3 tools/dump_solution.py gpurun_out/${TAG}_d_${v}_$c.json $c >> gpurun_out/${TAG}_dump.log 2>&1 || exit 1
done; done
for v in $VARS; do [ $v = $REF ] && continue; for c in ${DUMP:-B D C}; do
  python3 tools/dump_solution.py --compare gpurun_out/${TAG}_d_${REF}_$c.json gpurun_out/${TAG}_d_${v}_$c.json > /dev/null || { echo "NOT BIT-EXACT $v $c"; exit 1; }
done; done
echo "bit-exact: $VARS"
ROUNDS=${ROUNDS:-2} timeout -k 10 700 bash tools/ab.sh "$VARS" "$CFGS" > gpurun_out/${TAG}_ab.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${TAG}_ab.log
