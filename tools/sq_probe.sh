#!/bin/bash
# SQ counters of the walk kernel on the latency probe's single hardest point (GPU box):
#   tools/sq_probe.sh TAG   -> gpurun_out/TAG_sq{1,2}/...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-sq}
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/${TAG}_sq1 -o sq --output-format csv -- python3 tools/latency_probe.py hardest1 > gpurun_out/${TAG}_sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/${TAG}_sq2 -o sq --output-format csv -- python3 tools/latency_probe.py hardest1 > gpurun_out/${TAG}_sq2.log 2>&1
