#!/bin/bash
# (1) tail A/B base6 vs pkreuse (hashes, B / C timings, latency probe); (2) 3D census: D_cube64
# timings and config-D SQ passes of the 3D probe builds; (3) DIAG sections on D_cube64.
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
bash tools/r5h_call.sh r5i "base6 pkreuse" || exit 1
ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "base6 p3d1 p3d2 p3d16 p3d32" "D_cube64" > gpurun_out/r5i_ab3d.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/r5i_ab3d.log
for v in base6 p3d1 p3d2 p3d16 p3d32; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 300 python3 tools/collect_sq.py r5i_$v D > gpurun_out/r5i_${v}_sq.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r5i_${v}_walk_sq.json'));c=d['counters'];print('$v VALU %.1fM SALU %.1fM t %.3f ms issue %.3f' % (c['SQ_INSTS_VALU']/1e6, c['SQ_INSTS_SALU']/1e6, d['kernel_s']*1e3, d['valu_issue_frac']))"
done
WOS_LIB_PATH=$L/libwos_diag.so timeout -k 10 200 python3 tools/time_configs.py D_cube64 > gpurun_out/r5i_diag_D.log 2>&1 || exit 1
grep "diag" gpurun_out/r5i_diag_D.log | head -12
