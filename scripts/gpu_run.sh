# usage: bash scripts/gpu_run.sh TAG  -- GPU parity tests, full bench line, then kernel-trace + PMC profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh $T; rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_summary.py $T gpurun_out/${T}_pmc_summary.json "$(python -c 'import sys; sys.path.insert(0,"."); from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi; print(_abi.lib().hc_trifocal_version().decode())')" > /dev/null; echo "summary rc=$?"
cp gpurun_out/${T}_trace/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
