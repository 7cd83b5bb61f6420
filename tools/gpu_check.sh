#!/bin/bash
# GPU check (GPU box, repo root): the engine pin against the reference's own outputs first
# (fast feedback), then the whole -m gpu suite and smoke(), then the default bench line.
# Outputs in gpurun_out/<tag>_*.        tools/gpu_check.sh TAG
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_pin.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pin.log 2>&1 || { tail -30 gpurun_out/${TAG}_pin.log; exit 1; }
tail -3 gpurun_out/${TAG}_pin.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
