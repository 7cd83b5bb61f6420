#!/bin/bash
# Cost probes (GPU box, repo root).
#   tools/cost_probes.sh TAG                  round 5's first set: the fast-Bessel build against its exact-only
#                                             twin (solution hashes on B, D, C must match), timings of those and
#                                             of the WOS_PROBE 1/2/4 duplication builds, their SQ_INSTS_VALU (one
#                                             issue pass per variant), and the HBM-accounting builds'
#                                             FETCH_SIZE / WRITE_SIZE passes (config B)
#   tools/cost_probes.sh TAG "base probe8 ..." [CFG]   timings (B, C; D_cube64 and D_cube128 for CFG D) and one
#                                             SQ issue pass (CFG, default B) per named variant
# Variants: tools/build_variant.sh NAME "-DWOS_PROBE=k" (never shipped).
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
if [ -n "$2" ]; then
  CFG=${3:-B}; CASES="B_karman64k C_dirichlet512"; [ $CFG = D ] && CASES="D_cube64 D_cube128"
  ROUNDS=2 timeout -k 10 500 bash tools/ab.sh "$2" "$CASES" > gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  python3 tools/ab_summary.py gpurun_out/${TAG}_ab.log
  for v in $2; do
    WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 300 python3 tools/collect_sq.py ${TAG}_$v $CFG > gpurun_out/${TAG}_${v}_sq.log 2>&1 || exit 1
  done
  echo done
  exit 0
fi
for v in nofbes fbes; do for c in B D C; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 200 python3 tools/dump_solution.py gpurun_out/${TAG}_d_${v}_$c.json $c >> gpurun_out/${TAG}_dump.log 2>&1 || exit 1
done; done
for c in B D C; do python3 tools/dump_solution.py --compare gpurun_out/${TAG}_d_nofbes_$c.json gpurun_out/${TAG}_d_fbes_$c.json || { echo "NOT BIT-EXACT fbes $c"; exit 1; }; done
ROUNDS=2 timeout -k 10 500 bash tools/ab.sh "nofbes fbes probe1 probe2 probe4" "B_karman64k C_dirichlet512" > gpurun_out/${TAG}_ab.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${TAG}_ab.log
for v in nofbes fbes probe1 probe2 probe4; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 300 python3 tools/collect_sq.py ${TAG}_$v B > gpurun_out/${TAG}_${v}_sq.log 2>&1 || exit 1
done
for v in acct_base acct_notex acct_norec acct_nospread; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 400 python3 tools/collect_traffic.py ${TAG}_$v B > gpurun_out/${TAG}_${v}_traffic.log 2>&1 || exit 1
done
echo done
