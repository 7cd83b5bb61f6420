#!/bin/bash
# Round-5 GPU call (GPU box, repo root): the -m gpu suite, then an A/B of variant libraries
# on the named configs (timings only; bit-exactness of the variants by solution hashes on D
# and B), then the default bench line.       tools/r5_call.sh TAG "base v1 v2" "cfg1 cfg2"
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1; VARS=$2; CFGS=$3
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$VARS" ]; then
  REF=${VARS%% *}
  for v in $VARS; do for c in D B; do
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 200 python3 tools/dump_solution.py gpurun_out/${TAG}_d_${v}_$c.json $c >> gpurun_out/${TAG}_dump.log 2>&1 || exit 1
  done; done
  for v in $VARS; do [ $v = $REF ] && continue; for c in D B; do
    python3 tools/dump_solution.py --compare gpurun_out/${TAG}_d_${REF}_$c.json gpurun_out/${TAG}_d_${v}_$c.json > /dev/null || { echo "NOT BIT-EXACT $v $c"; exit 1; }
  done; done
  echo "bit-exact: $VARS"
  ROUNDS=${ROUNDS:-2} timeout -k 10 600 bash tools/ab.sh "$VARS" "$CFGS" > gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  python3 tools/ab_summary.py gpurun_out/${TAG}_ab.log 2>/dev/null || cat gpurun_out/${TAG}_ab.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && cat gpurun_out/${TAG}_bench.json
