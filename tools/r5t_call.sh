#!/bin/bash
# grid-wide tail spreading: the same kernel with the hand-overs off at run time (gspoff)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 500 bash tools/ab_latency.sh "head gsp1 gspoff" > gpurun_out/r5t_latency.log 2>&1 || exit 1
python3 tools/ab_latency_summary.py gpurun_out/r5t_latency.log
