#!/bin/bash
# tail A/B (GPU box): solution hashes, then the latency probe (stride-8 shard, hardest points)
# and the config timings of the variants.      tools/r5h_call.sh TAG "base v1"
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1; VARS=$2
bash tools/r5e_call.sh $TAG "$VARS" "B_karman64k C_dirichlet512" || exit 1
ROUNDS=2 timeout -k 10 500 bash tools/ab_latency.sh "$VARS" > gpurun_out/${TAG}_lat.log 2>&1 || exit 1
python3 tools/ab_latency_summary.py gpurun_out/${TAG}_lat.log 2>/dev/null || cat gpurun_out/${TAG}_lat.log
