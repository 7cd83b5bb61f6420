#!/bin/bash
# GPU suite + bench on the shipped lib, then the 3D fold-chunk A/B
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/r5_call.sh r5o "" "" || exit 1
bash tools/r5e_call.sh r5o2 "fc16 fc8 fc4" "D_cube128 E_cube96"
