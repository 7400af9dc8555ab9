# round 5 validation of the shipped build, part 2: kernel trace + PMC passes of
# the bench (scripts/profile.sh) and the dataset spread (scripts/datasets.py)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5v}
L=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
bash scripts/profile.sh $T; rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_summary.py $T gpurun_out/${T}_pmc_summary.json "$(python -c 'import sys; sys.path.insert(0,"."); from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi; print(_abi.lib().hc_trifocal_version().decode())')" > /dev/null; echo "summary rc=$?"
cp gpurun_out/${T}_trace/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
timeout -k 10 400 python scripts/datasets.py $L/libhc_trifocal_luwork.so > gpurun_out/${T}_datasets.jsonl; rc=$?; cat gpurun_out/${T}_datasets.jsonl; exit $rc
