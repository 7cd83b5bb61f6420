#!/bin/bash
# the new lone-walk parity test + the DIAG probe naming the slowest first-ball point
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lone_walks" --timeout 240 --timeout-method thread > gpurun_out/r3z_lone_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3z_lone_tests.log; [ $rc -eq 0 ] || exit $rc
WOS_LIB_PATH=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var/libwos_diag.so timeout -k 10 200 python3 tools/latency_probe.py > gpurun_out/r3z_diagfb.log 2>&1
