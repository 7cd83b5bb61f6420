#!/bin/bash
# grid-wide tail spreading, probers restricted by their SIMD's busy waves (0 / 1 / unrestricted)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/r5e_call.sh r5s "head gsp0 gsp1 gspa" "B_karman64k C_dirichlet512" || exit 1
ROUNDS=2 timeout -k 10 500 bash tools/ab_latency.sh "head gsp0 gsp1 gspa" > gpurun_out/r5s_latency.log 2>&1 || exit 1
python3 tools/ab_latency_summary.py gpurun_out/r5s_latency.log
