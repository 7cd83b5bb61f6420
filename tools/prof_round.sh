#!/bin/bash
# Measurement bundle of a round (GPU box, repo root): GPU parity tests, the default
# bench line, rocprofv3 kernel-trace stats of a short bench, PMC traffic passes and
# one SQ pass of the walk kernel.  Outputs under gpurun_out/<tag>_*.
#   tools/prof_round.sh TAG
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-projection-wall > gpurun_out/${TAG}_kt.log 2>&1 &&
timeout -k 10 600 python3 tools/collect_traffic.py ${TAG} > gpurun_out/${TAG}_traffic.log 2>&1 &&
timeout -k 10 300 python3 tools/collect_sq.py ${TAG} > gpurun_out/${TAG}_sq.log 2>&1
