set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/t_v9.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_v9.json 2> gpurun_out/bench_v9.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt9 -o kt9 --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kt9.log 2>&1
timeout -k 10 900 python3 tools/collect_traffic.py r1 > gpurun_out/traffic_v9.log 2>&1
