#!/bin/bash
# VALU census by cost probes (GPU box): timing and SQ issue pass of the base build and of each
# WOS_PROBE duplication build on config B.          tools/r5f_call.sh TAG "base p1 p2 ..."
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1; VARS=$2
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "$VARS" "B_karman64k" > gpurun_out/${TAG}_ab.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${TAG}_ab.log
for v in $VARS; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 300 python3 tools/collect_sq.py ${TAG}_$v B > gpurun_out/${TAG}_${v}_sq.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_walk_sq.json'));c=d['counters'];print('$v VALU %.1fM SALU %.1fM t %.3f ms issue %.3f' % (c['SQ_INSTS_VALU']/1e6, c['SQ_INSTS_SALU']/1e6, d['kernel_s']*1e3, d['valu_issue_frac']))"
done
