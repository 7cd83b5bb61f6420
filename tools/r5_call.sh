cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
L=$PWD/neural-monte-carlo-fluid-simulation_amd/lib/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5a_tests.log; [ $rc -eq 0 ] || exit $rc
for v in fbbase fbpack; do for c in D A; do
  WOS_LIB_PATH=$L/libwos_$v.so timeout -k 10 200 python3 tools/dump_solution.py gpurun_out/r5a_d_${v}_$c.json $c --shard8 >> gpurun_out/r5a_dump.log 2>&1 || exit 1
done; done
for c in D A; do python3 tools/dump_solution.py --compare gpurun_out/r5a_d_fbbase_$c.json gpurun_out/r5a_d_fbpack_$c.json || exit 1; done
ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "fbbase fbpack" "D_cube128 D_cube64" > gpurun_out/r5a_ab_fbpack.log 2>&1; cat gpurun_out/r5a_ab_fbpack.log
