#!/bin/bash
# The shipped library's bundle (GPU box, repo root), in two gpurun calls so each fits the
# call limit:
#   tools/bundle.sh TAG check   engine pin, -m gpu suite, smoke, default bench line
#                               (tools/gpu_check.sh), then the PMC bundle of every config
#                               (tools/measure_configs.sh: kernel trace, traffic, SQ passes)
#   tools/bundle.sh TAG bench   every config's bench line with its CPU baseline
#                               (tools/bench_configs.sh); run after the PMC JSONs are copied
#                               into profiles/, so the lines carry traffic and valu_issue
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1
case $2 in
  check) bash tools/gpu_check.sh $TAG && bash tools/measure_configs.sh $TAG ;;
  bench) bash tools/bench_configs.sh $TAG ;;
  *) echo "usage: tools/bundle.sh TAG check|bench"; exit 2 ;;
esac
