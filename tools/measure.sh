#!/bin/bash
# Measurement bundle of the shipped library (GPU box, repo root): rocprofv3 kernel-trace stats
# of a short bench (weak workload only), the PMC traffic passes and the SQ passes (issue,
# instruction mix) of the walk kernel.  Outputs under gpurun_out/<tag>_*.        tools/measure.sh TAG
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-projection-wall --no-strong > gpurun_out/${TAG}_kt.log 2>&1 &&
timeout -k 10 600 python3 tools/collect_traffic.py ${TAG} > gpurun_out/${TAG}_traffic.log 2>&1 &&
timeout -k 10 300 python3 tools/collect_sq.py ${TAG} > gpurun_out/${TAG}_sq.log 2>&1 &&
timeout -k 10 300 python3 tools/collect_sq.py ${TAG} B mix > gpurun_out/${TAG}_mix.log 2>&1 &&
timeout -k 10 300 python3 tools/collect_sq.py ${TAG} B mix2 > gpurun_out/${TAG}_mix2.log 2>&1
