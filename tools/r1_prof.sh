# Round-1 measurement bundle (run on the GPU box from the repo root):
#   GPU parity tests, default bench line, rocprofv3 kernel-trace stats of the bench,
#   PMC traffic passes of the walk kernel.  Outputs under gpurun_out/.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_kt.log 2>&1
timeout -k 10 900 python3 tools/collect_traffic.py ${TAG} > gpurun_out/${TAG}_traffic.log 2>&1
