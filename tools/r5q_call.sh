#!/bin/bash
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/r5e_call.sh r5q "fold1 fold4p" "B_karman64k C_dirichlet512 D_cube128 E_cube96"
