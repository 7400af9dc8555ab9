# round 5 validation of the shipped build, part 1: GPU tests, the default bench
# line, the LU-work count of the same sources
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5v}
L=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so timeout -k 10 200 python scripts/lu_work.py > gpurun_out/${T}_lu_work.json; rc=$?; cat gpurun_out/${T}_lu_work.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json; exit $rc
