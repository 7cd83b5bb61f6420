#!/bin/bash
# GPU suite on the shipped build, then A/B of the stratified-sample kernel split (lhs*), the
# fold unroll (fu8) against the previous build (pre), then the DIAG first-ball statistics
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3x_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_generic.sh ab6 "pre lhs solo lhs5 lhs43 fu8" &&
WOS_LIB_PATH=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var/libwos_diag.so timeout -k 10 120 python3 tools/time_configs.py B_karman64k > gpurun_out/diag2.log 2>&1
