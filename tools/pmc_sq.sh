#!/bin/bash
# SQ instruction-mix / stall passes of one configuration (GPU box):
#   tools/pmc_sq.sh TAG CONFIG     -> gpurun_out/TAG_sq{1,2}/
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; CFG=$2
timeout -s KILL 90 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/${TAG}_sq1 -o sq1 --output-format csv -- python3 tools/run_config.py $CFG 2 > gpurun_out/${TAG}_sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --kernel-trace -d gpurun_out/${TAG}_sq2 -o sq2 --output-format csv -- python3 tools/run_config.py $CFG 2 > gpurun_out/${TAG}_sq2.log 2>&1
