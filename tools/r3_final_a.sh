#!/bin/bash
# Final measurement bundle, part A (GPU box, repo root): the -m gpu suite, smoke(), the
# rocprofv3 kernel-trace stats of a short bench, the PMC traffic passes and the SQ pass of
# the walk kernel on the shipped build.  Outputs under gpurun_out/<tag>_*.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r3z}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-projection-wall --no-strong > gpurun_out/${TAG}_kt.log 2>&1 &&
timeout -k 10 600 python3 tools/collect_traffic.py ${TAG} > gpurun_out/${TAG}_traffic.log 2>&1 &&
timeout -k 10 300 python3 tools/collect_sq.py ${TAG} > gpurun_out/${TAG}_sq.log 2>&1
