#!/bin/bash
# grid-wide tail spreading: bit-exactness and timing against the workgroup-only build, the
# latency probe, then the scheduling-switch test (64 combinations)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/r5e_call.sh r5r "head gsp" "B_karman64k C_dirichlet512" || exit 1
ROUNDS=2 timeout -k 10 400 bash tools/ab_latency.sh "head gsp" > gpurun_out/r5r_latency.log 2>&1 || exit 1
python3 tools/ab_latency_summary.py gpurun_out/r5r_latency.log 2>/dev/null || tail -20 gpurun_out/r5r_latency.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5r_tests.log 2>&1; tail -3 gpurun_out/r5r_tests.log
