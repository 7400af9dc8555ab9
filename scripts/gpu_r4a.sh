# round 4, first lease: every GPU test, the bench line, trace + PMC of the same
# build (scripts/profile.sh), and the LU-work count of the same sources
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r4g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh ${T} || exit 1
HC_TRIFOCAL_LIB=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_luwork.so timeout -k 10 120 python scripts/lu_work.py > gpurun_out/${T}_lu_work.json; rc=$?; cat gpurun_out/${T}_lu_work.json; exit $rc
