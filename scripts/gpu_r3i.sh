# round-3 final build (spill-free stage loop + adaptive slice quantum): every GPU test,
# the dense re-solve count of the forcing test's input, the full bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3i_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3i_pytest.log; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so timeout -k 10 120 python scripts/lu_work.py --scaled > gpurun_out/r3i_lu_work_scaled.json 2>&1; rc=$?; cat gpurun_out/r3i_lu_work_scaled.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3i_bench.json 2> gpurun_out/r3i_bench.err; rc=$?; cat gpurun_out/r3i_bench.json; exit $rc
