#!/bin/bash
# Round-3 GPU check (GPU box, repo root): the whole -m gpu suite, then the default bench
# line.  Outputs in gpurun_out/<tag>_*.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
