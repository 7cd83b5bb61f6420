#!/bin/bash
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/r5e_call.sh r5p "fold1 fold4" "B_karman64k C_dirichlet512 D_cube128 E_cube96" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p_tests.log 2>&1; tail -3 gpurun_out/r5p_tests.log
