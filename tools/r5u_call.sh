#!/bin/bash
# round-5 check of the shipped library: the grid-spread latency A/B, then engine pin, GPU suite,
# smoke and the default bench line (tools/gpu_check.sh)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
ROUNDS=2 timeout -k 10 400 bash tools/ab_latency.sh "head gsp1 gspoff" > gpurun_out/r5t_latency.log 2>&1 || exit 1
python3 tools/ab_latency_summary.py gpurun_out/r5t_latency.log
bash tools/gpu_check.sh r5u
