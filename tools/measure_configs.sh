#!/bin/bash
# PMC bundle of the walk kernel on every bench config (GPU box, repo root): the rocprofv3
# kernel-trace stats of config B's bench, then per config (default "B C D E") the traffic
# passes (FETCH_SIZE, WRITE_SIZE), the SQ issue pass and the instruction-mix passes, combined into the
# calibrated VALU issue fraction with this box's per-type issue costs (tools/mb_latency issue).
# Outputs gpurun_out/<tag>_*; copy the JSONs to profiles/ so bench.py reports them.
#   tools/measure_configs.sh TAG ["B C D E"]
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
TAG=$1; CFGS=${2:-"B C D E"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-projection-wall --no-strong > gpurun_out/${TAG}_kt.log 2>&1 || exit 1
# the issue cost of each VALU instruction type on this box (calibrates the SQ passes' issue fraction)
timeout -k 10 120 ./tools/mb_latency issue > gpurun_out/${TAG}_mb_issue.json 2> gpurun_out/${TAG}_mb_issue.err || exit 1
for c in $CFGS; do
  t=${TAG}_$c; [ $c = B ] && t=$TAG
  timeout -k 10 600 python3 tools/collect_traffic.py $t $c > gpurun_out/${t}_traffic.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/collect_sq.py $t $c > gpurun_out/${t}_sq.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/collect_sq.py $t $c mix > gpurun_out/${t}_mix.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/collect_sq.py $t $c mix2 > gpurun_out/${t}_mix2.log 2>&1 || exit 1
  python3 tools/collect_sq.py combine $TAG $c gpurun_out/${TAG}_mb_issue.json >> gpurun_out/${TAG}_issue.log 2>&1 || exit 1
done
