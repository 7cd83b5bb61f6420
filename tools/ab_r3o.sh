cd /root/repo && export TMPDIR=/tmp
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
WOS_LIB_PATH=$L/libwos_base.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/d_base.npz B --shard8 > gpurun_out/r3o_dump.log 2>&1 &&
WOS_LIB_PATH=$L/libwos_all.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/d_all.npz B --shard8 >> gpurun_out/r3o_dump.log 2>&1 &&
WOS_LIB_PATH=$L/libwos_pk.so timeout -k 10 120 python3 tools/dump_solution.py gpurun_out/d_pk.npz B --shard8 >> gpurun_out/r3o_dump.log 2>&1 &&
python3 tools/dump_solution.py --compare gpurun_out/d_base.npz gpurun_out/d_all.npz >> gpurun_out/r3o_dump.log 2>&1 &&
python3 tools/dump_solution.py --compare gpurun_out/d_base.npz gpurun_out/d_pk.npz >> gpurun_out/r3o_dump.log 2>&1 &&
ROUNDS=2 timeout -k 10 600 bash tools/ab_latency.sh "base all sb rt dt pk" > gpurun_out/r3o_ab.log 2>&1 &&
WOS_LIB_PATH=$L/libwos_diag.so timeout -k 10 200 python tools/latency_probe.py > gpurun_out/r3o_lat_diag.jsonl 2> gpurun_out/r3o_lat_diag.err
