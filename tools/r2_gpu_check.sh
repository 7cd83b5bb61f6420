#!/bin/bash
# Round-2 GPU check (GPU box, repo root): the whole -m gpu suite, then the default
# bench line and the 8-GPU configs' single-GPU bench lines.  Outputs in gpurun_out/.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
timeout -k 10 300 python bench.py --config D --steps 5 --warmup 1 > gpurun_out/${TAG}_bench_D.json 2> gpurun_out/${TAG}_bench_D.err &&
timeout -k 10 300 python bench.py --config E --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_E.json 2> gpurun_out/${TAG}_bench_E.err &&
timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 > gpurun_out/${TAG}_bench_C.json 2> gpurun_out/${TAG}_bench_C.err
