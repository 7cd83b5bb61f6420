#!/bin/bash
# GPU suite + bench line on the shipped build, the latency probe of the build (cur) and
# the DIAG sections of its walk kernel (diag), TAG-prefixed under gpurun_out/
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
TAG=${1:-r3y}
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
WOS_LIB_PATH=$L/libwos_cur.so timeout -k 10 200 python3 tools/latency_probe.py > gpurun_out/${TAG}_probe.log 2>/dev/null &&
WOS_LIB_PATH=$L/libwos_diag.so timeout -k 10 120 python3 tools/time_configs.py B_karman64k > gpurun_out/${TAG}_diag.log 2>&1 &&
WOS_LIB_PATH=$L/libwos_diag.so timeout -k 10 200 python3 tools/latency_probe.py hardest1 > gpurun_out/${TAG}_diag_h1.log 2>&1
