#!/bin/bash
# Kernel-trace stats of one config under an environment switch (GPU box, repo root):
#   tools/kt_env.sh TAG VAR "v1 v2" CONFIG   ->  gpurun_out/TAG_VAR=v_stats.csv
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; VAR=$2; CFG=$4
mkdir -p gpurun_out
for v in $3; do
  env "$VAR=$v" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt_$v -o kt --output-format csv \
    -- python3 tools/time_configs.py $CFG > gpurun_out/${TAG}_kt_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/${TAG}_kt_$v -name "kt_kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_${VAR}=${v}_stats.csv
  rm -rf gpurun_out/${TAG}_kt_$v
done
