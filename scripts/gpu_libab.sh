# usage: bash scripts/gpu_libab.sh TAG LIB_A LIB_B ...  -- GPU parity tests on the default
# lib, then ubench (kernel ms, config 2) for each alternative build of the library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for L in "$@"; do
  HC_TRIFOCAL_LIB=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib/$L timeout -k 10 200 python scripts/ubench.py > gpurun_out/${T}_${L%.so}_$rep.json 2>gpurun_out/${T}_ub.err; rc=$?; [ $rc -eq 0 ] || { echo "ubench $L rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_${L%.so}_$rep.json'));print('$L', round(d['track_ms'],2), round(d['track1_ms'],3), round(d['cgesv_ns_per_solve'],3))"
done; done
if [ -f trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_phases.so ]; then
  HC_TRIFOCAL_LIB=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_phases.so timeout -k 10 200 python scripts/diag_phases.py > gpurun_out/${T}_phases.json; rc=$?; [ $rc -eq 0 ] || { echo "phases rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_phases.json'));[print(k, d[k]['per_stage_pair']) for k in d]"
fi
