#!/bin/bash
# One bench line per configuration with its CPU baseline (and, for the strong-scaled C, D, E,
# the stride-8 shard), plus the two-rank gloo rehearsal of the N-rank bench path, into
# gpurun_out/<tag>_bench_<cfg>.json (GPU box, repo root).     tools/bench_configs.sh TAG
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 240 python -u -m pytest tests/test_bench_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_bdist.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_B.json 2> gpurun_out/${TAG}_bench_B.err &&
timeout -k 10 240 python bench.py --config C --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_C.json 2> gpurun_out/${TAG}_bench_C.err &&
timeout -k 10 240 python bench.py --config D --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_D.json 2> gpurun_out/${TAG}_bench_D.err &&
timeout -k 10 300 python bench.py --config E --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_E.json 2> gpurun_out/${TAG}_bench_E.err &&
timeout -k 10 240 python bench.py --config A_robust --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_A_robust.json 2> gpurun_out/${TAG}_bench_A_robust.err &&
timeout -k 10 240 python bench.py --config A --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_A.json 2> gpurun_out/${TAG}_bench_A.err
